#!/bin/bash
# bf16 direct packing through the full-size / oracle tests, RCCL with the
# residency gate, step times (configs[4] with the in-cell bf16 backward)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
KCTC_BF16_DIRECT=1 $T 500 python -u -m pytest tests/test_fullsize_gpu.py tests/test_train_gpu.py tests/test_rnn_gpu.py -x -q -k "bf16 or cfg4" --timeout 300 --timeout-method thread > gpurun_out/bf16_full.log 2>&1
rc=$?; echo "bf16_full rc=$rc"; tail -2 gpurun_out/bf16_full.log; [ $rc -eq 0 ] || exit 1
KCTC_COMM_GATE=1 $T 300 python -u -m pytest tests/test_train_gpu.py -x -q -k "rccl" --timeout 250 --timeout-method thread > gpurun_out/rccl_gate.log 2>&1
rc=$?; echo "rccl_gate rc=$rc"; tail -2 gpurun_out/rccl_gate.log; [ $rc -eq 0 ] || exit 1
DIAGS="c4noio:X=0 c4io:KCTC_BF16_DIRECT=1" CFG=4 $T 300 bash scripts/gpu_diag.sh && DIAGS="base:X=0" $T 100 bash scripts/gpu_diag.sh
