#!/bin/bash
# H2D-inclusive pass: copy stream one step ahead vs the copy on the trainer's stream
set -o pipefail
mkdir -p gpurun_out
for tag in new old new2 old2; do
  extra=""; case $tag in old*) extra="BENCH_H2D_ON_COMPUTE=1";; esac
  env $extra timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline --no-loss-match > gpurun_out/h2d_$tag.log 2>&1 || { echo "FAILED $tag"; tail -3 gpurun_out/h2d_$tag.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/h2d_$tag.log').read().strip().splitlines()[-1])
print('$tag', d['value'], d['median_step_ms'], d['h2d_inclusive'])"
done
