#!/bin/bash
# per-phase recurrence trace of the default configuration (first fwd + bwd launch)
set -o pipefail
mkdir -p gpurun_out/tr2
export TMPDIR=/tmp
env $1 KCTC_REC_TRACE=gpurun_out/tr2 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-h2d-pass > gpurun_out/tr2.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr2.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr2/rec_fwd.bin gpurun_out/tr2/rec_bwd.bin
