#!/bin/bash
# gated projection probes, bit-identity test, then step times (forward without the per-wave stamps)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 100 python -u scripts/gate_probe.py off d1 d2 full > gpurun_out/gate_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; tail -8 gpurun_out/gate_probe.log; [ $rc -eq 0 ] || exit 1
$T 300 python -u -m pytest tests/test_fwd_gate_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fgate.log 2>&1
rc=$?; echo "fgate rc=$rc"; tail -3 gpurun_out/fgate.log; [ $rc -eq 0 ] || exit 1
DIAGS="base:X=0 gate:KCTC_FWD_GATE=1 base2:X=0 gate2:KCTC_FWD_GATE=1" $T 400 bash scripts/gpu_diag.sh || exit 1
TRACES="base:X=0 gate:KCTC_FWD_GATE=1" $T 300 bash scripts/gpu_trace_diag.sh
