#!/bin/bash
# GPU sweep: parity tests, then bench variants (env knobs of the trainer).
# usage: bash scripts/gpu_sweep.sh "ENV=.. ENV=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v$i.log 2>&1 || { echo BENCH_FAILED $cfg; tail -5 gpurun_out/bench_v$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_v$i.log').read().strip().splitlines()[-1]); print('$cfg |', d['value'], d['ms_per_step'], d['roofline']['families_ms_per_step'])"
done
