#!/bin/bash
# Bench variants only (no tests): usage bash scripts/gpu_sweep_nt.sh "ENV=.. ENV=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_v$i.log 2>&1 || { echo BENCH_FAILED $cfg; tail -5 gpurun_out/sweep_v$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_v$i.log').read().strip().splitlines()[-1]); f=d['roofline']['families_ms_per_step']; print('$cfg |', d['value'], d['ms_per_step'], 'fwd', f['rnn_fwd_rec'], 'bwd', f['rnn_bwd_rec'])"
done
