#!/bin/bash
# feature validations: bf16 direct packing (+ configs[4] A/B), 16-workgroup
# pinning (+ configs[2] A/B), residency-gated exchange, CU shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_bf16_direct_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/bf16d.log 2>&1
rc=$?; echo "bf16d rc=$rc"; tail -2 gpurun_out/bf16d.log
if [ $rc -eq 0 ]; then DIAGS="c4noio:X=0 c4io:KCTC_BF16_DIRECT=1" CFG=4 $T 300 bash scripts/gpu_diag.sh || exit 1; fi
KCTC_XCD6_HALF=1 $T 300 python -u -m pytest tests/test_xcd_pin_gpu.py -x -q -k "64 or 57" --timeout 250 --timeout-method thread > gpurun_out/pin_half.log 2>&1
rc=$?; echo "pin_half rc=$rc"; tail -2 gpurun_out/pin_half.log
if [ $rc -eq 0 ]; then DIAGS="c2base:X=0 c2half:KCTC_XCD6_HALF=1" CFG=2 $T 300 bash scripts/gpu_diag.sh || exit 1; fi
KCTC_COMM_GATE=1 $T 400 python -u -m pytest tests/test_cu_budget_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gate_ex.log 2>&1
rc=$?; echo "gate_ex rc=$rc"; tail -2 gpurun_out/gate_ex.log
[ $rc -eq 0 ] || exit 1
$T 120 python -u -m pytest tests/test_cu_partition_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/cupart.log 2>&1
echo "cupart rc=$?"; tail -2 gpurun_out/cupart.log
