#!/bin/bash
# round-4 measurement: bench + rocprofv3 stats + PMC traffic + timeline +
# recurrence phase traces (configs[1]), then configs[2] / [4] benches + stats;
# large raw traces are summarised and removed so that gpurun_out stays small
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_bench_prof.sh || exit 1
python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv 50 > gpurun_out/timeline.txt 2>&1 || true
mkdir -p gpurun_out/keep
find gpurun_out/prof -name "*kernel_stats*" -exec cp {} gpurun_out/keep/kernel_stats.csv \;
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
TRACES="base:X=0" timeout -k 10 150 bash scripts/gpu_trace_diag.sh > gpurun_out/trace_summary.txt 2>&1 || exit 1
bash scripts/gpu_cfg_prof.sh || exit 1
for c in 2 4; do find gpurun_out/prof_cfg$c -name "*kernel_stats*" -exec cp {} gpurun_out/keep/cfg${c}_kernel_stats.csv \; ; done
rm -rf gpurun_out/prof_cfg2 gpurun_out/prof_cfg4
ls gpurun_out gpurun_out/keep
