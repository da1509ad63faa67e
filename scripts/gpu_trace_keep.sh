#!/bin/bash
# one traced configs[N] step (KCTC_REC_TRACE): the raw phase stamps kept under gpurun_out/tr_keep
set -o pipefail
mkdir -p gpurun_out/tr_keep
KCTC_REC_TRACE=gpurun_out/tr_keep timeout -k 10 200 python bench.py --config ${CFG:-1} --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr_keep.log 2>&1 || { echo TRACE_FAILED; tail -3 gpurun_out/tr_keep.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr_keep/rec_fwd.bin gpurun_out/tr_keep/rec_bwd.bin | grep -v "shader clock"
