#!/bin/bash
# GPU sweep: parity tests, then bench variants of the recurrence hand-off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -x -q > gpurun_out/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for cfg in "0 4 16" "1 4 16" "0 8 16" "0 4 8" "0 16 16"; do
  set -- $cfg
  KCTC_SYNC=$1 KCTC_FWD_U=$2 KCTC_BWD_U=$3 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s$1_f$2_b$3.log 2>&1 || { echo BENCH_FAILED $cfg; tail -5 gpurun_out/bench_s$1_f$2_b$3.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_s$1_f$2_b$3.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['families_ms_per_step'])"
done
