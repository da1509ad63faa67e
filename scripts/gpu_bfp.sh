#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py -x -v -s -k "bf16 or gru1024" --timeout 200 --timeout-method thread > gpurun_out/bfp_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/bfp_tests.log; exit 1; }
grep -E "e-0|passed|failed" gpurun_out/bfp_tests.log | cut -c1-220 | tail -25
BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh - c4_bfp KCTC_X=0 c4_fp32p KCTC_BF16_PARTIALS=0
