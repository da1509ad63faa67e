#!/bin/bash
# Round-3 first check: the new GPU tests (CU budget, DP failed-step
# agreement, CTC frame groups), the default bench (loss match, rooflines) and
# the 2-rank host-transport bench on one GPU (the launcher).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_cu_budget_gpu.py tests/test_dp_gpu.py tests/test_ctc_gpu.py > gpurun_out/r03a_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03a_tests.log; exit 1; }
tail -2 gpurun_out/r03a_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r03a_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03a_bench.log; exit 1; }
tail -1 gpurun_out/r03a_bench.log
timeout -k 10 300 python bench.py --gpus 2 --dp-transport host --steps 5 --warmup 2 > gpurun_out/r03a_bench_dp2.log 2>&1 || { echo DP2_FAILED; tail -20 gpurun_out/r03a_bench_dp2.log; exit 1; }
tail -1 gpurun_out/r03a_bench_dp2.log
