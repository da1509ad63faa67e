#!/bin/bash
# the tests added in a round first (one process), then the whole GPU suite and a short default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/component_gradcheck.txt
timeout -k 10 600 python -u -m pytest ${NEW_TESTS:-tests/test_component_gpu.py tests/test_recipe_config.py tests/test_decode_gpu.py} -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { echo NEW_TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/new_tests.log | head -30; tail -5 gpurun_out/new_tests.log; exit 1; }
tail -1 gpurun_out/new_tests.log
[ -n "$NO_SUITE" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/qb.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/qb.log; exit 1; }
tail -1 gpurun_out/qb.log
