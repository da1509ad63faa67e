#!/bin/bash
# packed GEMM: numerics (GEMM + RNN/train tests), then timing with 256 and 128 tiles, then the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 120 python scripts/gemm_packed_bench.py > gpurun_out/gemm256.log 2>&1 || { echo GB_FAILED; tail -5 gpurun_out/gemm256.log; exit 1; }
grep TF gpurun_out/gemm256.log
KCTC_GEMM256=0 timeout -k 10 120 python scripts/gemm_packed_bench.py > gpurun_out/gemm128.log 2>&1 || { echo GB_FAILED; tail -5 gpurun_out/gemm128.log; exit 1; }
grep TF gpurun_out/gemm128.log
bash scripts/gpu_variants.sh - g256 KCTC_X=0 g128 KCTC_GEMM256=0
BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh - c4_256 KCTC_X=0 c4_128 KCTC_GEMM256=0
