#!/bin/bash
# v4 recurrence validation: parity tests, bench variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_egs.py -x -q > gpurun_out/tests_v4.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_v4.log; exit 1; }
tail -2 gpurun_out/tests_v4.log
for cfg in "KCTC_LOCAL=0" "KCTC_LOCAL=1" "KCTC_SIDE_BLOCKS=192" "KCTC_FWD_U=8" "KCTC_FWD_U=4"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { echo BENCH_FAILED $cfg; tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg |', d['value'], d['ms_per_step'], d['roofline']['families_ms_per_step'])"
done
