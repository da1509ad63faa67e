#!/bin/bash
# checkpoint: smoke, full bench (CPU baseline, H2D pass), rocprof stats +
# PMC traffic + timeline (the GPU suite ran in scripts/gpu_quick.sh), then
# configs[2] / configs[4] benches with stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_bench_prof.sh || exit 1
python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv 50 > gpurun_out/timeline.txt 2>&1 || true
bash scripts/gpu_cfg_prof.sh || exit 1
