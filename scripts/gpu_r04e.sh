#!/bin/bash
# gated projection probe + test, then step times and traces for the new backward cell
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 90 python -u scripts/gate_probe.py off d1 d2 full > gpurun_out/gp.log 2>&1; echo "probe rc=$?"; tail -5 gpurun_out/gp.log
grep -q "full .*same_as_off True" gpurun_out/gp.log || exit 0
$T 300 python -u -m pytest tests/test_fwd_gate_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fgate.log 2>&1
rc=$?; echo "fgate rc=$rc"; tail -3 gpurun_out/fgate.log; [ $rc -eq 0 ] || exit 1
DIAGS="base:X=0 gate:KCTC_FWD_GATE=1 base2:X=0 gate2:KCTC_FWD_GATE=1" $T 400 bash scripts/gpu_diag.sh && TRACES="gate:KCTC_FWD_GATE=1" $T 150 bash scripts/gpu_trace_diag.sh
