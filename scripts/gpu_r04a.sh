#!/bin/bash
# round-4 checks: backward IO waves and the gated forward projection
# (bit-identity, traces, step times), bf16 direct packing, cfg4 A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
KCTC_BWD_IOW=1 $T 400 python -u -m pytest tests/test_xcd_pin_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pin_iow.log 2>&1
rc=$?; echo "pin_iow rc=$rc"; tail -3 gpurun_out/pin_iow.log
[ $rc -eq 0 ] || exit 1
$T 300 python -u -m pytest tests/test_fwd_gate_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fgate.log 2>&1
rc=$?; echo "fgate rc=$rc"; tail -3 gpurun_out/fgate.log
[ $rc -eq 0 ] || exit 1
TRACES="base:X=0 iow:KCTC_BWD_IOW=1" $T 300 bash scripts/gpu_trace_diag.sh || exit 1
DIAGS="base:X=0 iow:KCTC_BWD_IOW=1 gate:KCTC_FWD_GATE=1 both:KCTC_BWD_IOW=1,KCTC_FWD_GATE=1 base2:X=0 both2:KCTC_BWD_IOW=1,KCTC_FWD_GATE=1" $T 500 bash scripts/gpu_diag.sh || exit 1
$T 300 python -u -m pytest tests/test_bf16_direct_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/bf16d.log 2>&1
echo "bf16d rc=$?"; tail -3 gpurun_out/bf16d.log
DIAGS="c4io:KCTC_BF16_DIRECT=1 c4noio:X=0" CFG=4 $T 300 bash scripts/gpu_diag.sh
