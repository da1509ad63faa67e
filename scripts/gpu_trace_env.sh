#!/bin/bash
# recurrence traces under env variants (no tests): bash scripts/gpu_trace_env.sh "ENV=.." ...
set -o pipefail
i=0
for cfg in "$@"; do
  i=$((i+1)); mkdir -p gpurun_out/tre$i
  env $cfg KCTC_REC_TRACE=gpurun_out/tre$i timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tre$i.log 2>&1 || { echo TRACE_FAILED $cfg; tail -5 gpurun_out/tre$i.log; exit 1; }
  echo "== $cfg"; python scripts/trace_rec.py gpurun_out/tre$i/rec_fwd.bin gpurun_out/tre$i/rec_bwd.bin | grep -v "skew\|clock"
done
