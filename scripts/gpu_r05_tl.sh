#!/bin/bash
# round 5: kernel timeline of one configs[1] step (critical path, compute-queue idle)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tl -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-loss-match --no-h2d-pass --no-profile > gpurun_out/prof_tl.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_tl.log; exit 1; }
tail -1 gpurun_out/prof_tl.log | cut -c1-200
f=$(find gpurun_out/prof_tl -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f 30 > gpurun_out/timeline_r05.txt 2>&1 || true
find gpurun_out/prof_tl -name "*kernel_stats*" -exec cp {} gpurun_out/kernel_stats_r05.csv \;
rm -rf gpurun_out/prof_tl
cat gpurun_out/timeline_r05.txt | tail -80
head -20 gpurun_out/kernel_stats_r05.csv | cut -c1-200
