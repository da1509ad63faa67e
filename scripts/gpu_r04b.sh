#!/bin/bash
# round-4 checks, part 2: configs[2] pinning (16-workgroup slots), the
# residency-gated exchange (CU-probe exchange, 2-rank DP), CU shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
KCTC_XCD6_HALF=1 $T 400 python -u -m pytest tests/test_xcd_pin_gpu.py -x -q -k "64 or 57" --timeout 300 --timeout-method thread > gpurun_out/pin_half.log 2>&1
rc=$?; echo "pin_half rc=$rc"; tail -3 gpurun_out/pin_half.log
[ $rc -eq 0 ] || exit 1
KCTC_COMM_GATE=1 $T 500 python -u -m pytest tests/test_cu_budget_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gate_ex.log 2>&1
rc=$?; echo "gate_ex rc=$rc"; tail -3 gpurun_out/gate_ex.log
[ $rc -eq 0 ] || exit 1
$T 200 python -u -m pytest tests/test_cu_partition_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/cupart.log 2>&1
echo "cupart rc=$?"; tail -3 gpurun_out/cupart.log
DIAGS="c2base:X=0 c2half:KCTC_XCD6_HALF=1" CFG=2 $T 300 bash scripts/gpu_diag.sh
