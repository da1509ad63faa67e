#!/bin/bash
# configs[4]: the streamed GEMMs (KCTC_STREAM_ALL=1) against the default
# (GEMMs after the recurrences), same box; each bench with its loss match
set -o pipefail
mkdir -p gpurun_out
for spec in base:X=1 sall:KCTC_STREAM_ALL=1; do
  tag=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 2 --no-cpu-baseline --no-h2d-pass > gpurun_out/c4_$tag.log 2>&1 || { echo "FAILED $tag"; tail -3 gpurun_out/c4_$tag.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/c4_$tag.log').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], d['loss_match']['pass'], r['secondary']['recurrence_step_us'], {k:v for k,v in r['families_ms_per_step'].items() if v>0.5})"
done
