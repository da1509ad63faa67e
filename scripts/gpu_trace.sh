#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tr0 gpurun_out/tr1
KCTC_REC_TRACE=gpurun_out/tr0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr0.log 2>&1 || { echo TRACE0_FAILED; tail -5 gpurun_out/tr0.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr0/rec_fwd.bin gpurun_out/tr0/rec_bwd.bin
KCTC_SYNC=1 KCTC_REC_TRACE=gpurun_out/tr1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr1.log 2>&1 || { echo TRACE1_FAILED; tail -5 gpurun_out/tr1.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr1/rec_fwd.bin
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_def.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/bench_def.log; exit 1; }
tail -1 gpurun_out/bench_def.log
