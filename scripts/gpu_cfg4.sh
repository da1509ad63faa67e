#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config 4 > gpurun_out/bench_cfg4.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_cfg4.log; exit 1; }
tail -1 gpurun_out/bench_cfg4.log
