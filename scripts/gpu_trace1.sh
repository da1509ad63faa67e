#!/bin/bash
# recurrence phase trace of one configs[1] step (default settings)
set -o pipefail
mkdir -p gpurun_out/tr0
KCTC_REC_TRACE=gpurun_out/tr0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr0.log 2>&1 || { echo TRACE0_FAILED; tail -5 gpurun_out/tr0.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr0/rec_fwd.bin gpurun_out/tr0/rec_bwd.bin
