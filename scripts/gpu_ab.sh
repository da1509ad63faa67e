#!/bin/bash
# same-box A/B of environment switches on configs[${CFG:-1}]: AB="tag:ENV=V,ENV2=V ..." (each twice, interleaved)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for spec in $AB; do
    tag=${spec%%:*}; envs=${spec#*:}
    env ${envs//,/ } timeout -k 10 300 python bench.py --config ${CFG:-1} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-loss-match --no-h2d-pass > gpurun_out/ab_${tag}_$round.log 2>&1 || { echo "FAILED $tag"; tail -3 gpurun_out/ab_${tag}_$round.log; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab_${tag}_$round.log').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], {k:v for k,v in r['families_ms_per_step'].items() if k in ('bwd_data_stream','fwd_proj_rows','rnn_bwd_rec','rnn_fwd_rec')})"
  done
done
