#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/n8_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/n8_tests.log; exit 1; }
tail -1 gpurun_out/n8_tests.log
BENCH_ARGS="--N 8" bash scripts/gpu_variants.sh - n8 KCTC_X=0 && BENCH_ARGS="--N 4" bash scripts/gpu_variants.sh - n4 KCTC_X=0 && bash scripts/gpu_variants.sh - n16 KCTC_X=0
