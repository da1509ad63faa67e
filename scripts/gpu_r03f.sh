#!/bin/bash
# Round-3 checkpoint after the XCD-pinned backward: whole GPU suite, smoke,
# bench + rocprof + PMC passes, timeline, then configs[2]/[4] stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit 1
bash scripts/gpu_cfg_prof.sh || exit 1
KCTC_XCD6=0 KCTC_XCD6F=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/bench_unpinned.log 2>&1 || { echo UNPINNED_FAILED; tail -5 gpurun_out/bench_unpinned.log; exit 1; }
tail -1 gpurun_out/bench_unpinned.log | cut -c1-300
