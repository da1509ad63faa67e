#!/bin/bash
# Round-3 checkpoint: whole GPU suite, smoke, bench + rocprof + PMC passes,
# timeline; then the all-fp32 MFMA path (KCTC_GEMM=f32, v4 recurrences) beside it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit 1
KCTC_GEMM=f32 KCTC_FWD_REC=4 KCTC_BWD_REC=4 timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2d-pass > gpurun_out/bench_fp32path.log 2>&1 || { echo FP32PATH_FAILED; tail -20 gpurun_out/bench_fp32path.log; exit 1; }
tail -1 gpurun_out/bench_fp32path.log | cut -c1-400
