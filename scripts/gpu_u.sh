#!/bin/bash
# v4 U sweep: parity (rnn) under each forward U, trace + bench per U.
set -o pipefail
mkdir -p gpurun_out
for U in 16 8 4; do
  KCTC_FWD_U=$U timeout -k 10 300 python -m pytest tests/test_rnn_gpu.py -x -q > gpurun_out/tests_u$U.log 2>&1 || { echo TESTS_FAILED U=$U; tail -30 gpurun_out/tests_u$U.log; exit 1; }
  mkdir -p gpurun_out/tru$U
  KCTC_FWD_U=$U KCTC_REC_TRACE=gpurun_out/tru$U timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tru$U.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tru$U.log; exit 1; }
  python scripts/trace_rec.py gpurun_out/tru$U/rec_fwd.bin
  KCTC_FWD_U=$U timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_u$U.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/bench_u$U.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_u$U.log').read().strip().splitlines()[-1]); print('U=$U |', d['value'], d['ms_per_step'], d['roofline']['families_ms_per_step'])"
done
