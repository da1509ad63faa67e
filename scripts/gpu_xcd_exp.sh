#!/bin/bash
# Experiment: backward recurrence with each (direction, row group) on one XCD
# (KCTC_XCD6=1: plain stores / L2 hand-off) vs the sc1 protocol, both without
# the streamed dx GEMM (XCD-slot launches do not stream).
set -o pipefail
mkdir -p gpurun_out/xa gpurun_out/xb
export TMPDIR=/tmp
KCTC_BWD_STREAM=0 KCTC_REC_TRACE=gpurun_out/xa timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-h2d-pass --no-loss-match > gpurun_out/xa.log 2>&1 || { echo A_FAILED; tail -5 gpurun_out/xa.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/xa.log').read().strip().splitlines()[-1]);print('A', d['value'], d['roofline']['secondary']['recurrence_step_us'])"
python scripts/trace_rec.py gpurun_out/xa/rec_bwd.bin
KCTC_XCD6=1 KCTC_BWD_STREAM=0 KCTC_REC_TRACE=gpurun_out/xb timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-h2d-pass > gpurun_out/xb.log 2>&1 || { echo B_FAILED; tail -5 gpurun_out/xb.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/xb.log').read().strip().splitlines()[-1]);print('B', d['value'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'], d['loss_match']['grad_sketch_err'])"
python scripts/trace_rec.py gpurun_out/xb/rec_bwd.bin
