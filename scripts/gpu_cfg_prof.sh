#!/bin/bash
# rocprofv3 kernel stats of configs[2] and configs[4] benches (secondary configurations)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 2 4; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_cfg$c.log 2>&1 || { echo BENCH_FAILED $c; tail -20 gpurun_out/bench_cfg$c.log; exit 1; }
  tail -1 gpurun_out/bench_cfg$c.log | cut -c1-300
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-h2d-pass > gpurun_out/prof_cfg$c.log 2>&1 || { echo PROF_FAILED $c; tail -20 gpurun_out/prof_cfg$c.log; exit 1; }
done
find gpurun_out/prof_cfg2 gpurun_out/prof_cfg4 -name "*kernel_stats*"
