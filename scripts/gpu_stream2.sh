#!/bin/bash
# streamed GEMMs over row groups and in bf16: parity tests, then benches of configs[1], [2], [4]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_rnn_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s2_tests.log; exit 1; }
tail -1 gpurun_out/s2_tests.log
bash scripts/gpu_variants.sh - c1 KCTC_X=0 || exit 1
BENCH_ARGS="--config 2" bash scripts/gpu_variants.sh - c2 KCTC_X=0 c2_nostream "KCTC_FWD_STREAM=0 KCTC_BWD_STREAM=0" || exit 1
BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh - c4 KCTC_X=0 c4_nostream KCTC_BF16_STREAM=0
