#!/bin/bash
# HIP runtime API trace of a short bench (host-side gaps between the forward and the backward)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace -d gpurun_out/api -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-loss-match --no-h2d-pass --no-profile > gpurun_out/api.log 2>&1 || { echo API_FAILED; tail -5 gpurun_out/api.log; exit 1; }
find gpurun_out/api -name "*.csv" | head
