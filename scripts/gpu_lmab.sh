#!/bin/bash
# does the loss-match pass (a second Nnet before the timed passes) change the timed rate?
set -o pipefail
mkdir -p gpurun_out
for tag in lm1 nolm lm2; do
  extra=""; [ $tag = nolm ] && extra="--no-loss-match"
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-h2d-pass $extra > gpurun_out/lmab_$tag.log 2>&1 || { echo "FAILED $tag"; tail -3 gpurun_out/lmab_$tag.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/lmab_$tag.log').read().strip().splitlines()[-1])
print('$tag', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['secondary'].get('profiled_pass'))"
done
