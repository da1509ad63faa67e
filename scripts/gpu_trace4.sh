#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tr4
KCTC_REC_TRACE=gpurun_out/tr4 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr4.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr4.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr4/rec_fwd.bin gpurun_out/tr4/rec_bwd.bin
