#!/bin/bash
# whole GPU suite, then configs[1], [2], [4] benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/gpu_variants.sh - c1 KCTC_X=0 || exit 1
BENCH_ARGS="--config 2" bash scripts/gpu_variants.sh - c2 KCTC_X=0 || exit 1
BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh - c4 KCTC_X=0
