#!/bin/bash
# checkpoint: whole GPU suite, smoke, full bench (CPU baseline, H2D pass),
# rocprof stats + PMC traffic + timeline, configs[2] / configs[4] with stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/gpu_bench_prof.sh || exit 1
python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv 50 > gpurun_out/timeline.txt 2>&1 || true
bash scripts/gpu_cfg_prof.sh || exit 1
