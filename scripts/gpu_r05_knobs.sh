#!/bin/bash
# round 5: side-stream / dx-stream block budgets (configs[1]), one short bench each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-loss-match --no-h2d-pass > gpurun_out/kn_$tag.log 2>&1 || { echo "KN_FAILED $tag"; tail -3 gpurun_out/kn_$tag.log; return 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/kn_$tag.log').read().strip().splitlines()[-1]);r=d['roofline'];f=r['families_ms_per_step']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], 'bwd_data_stream', f.get('bwd_data_stream'), 'bwd_w', f.get('gemm_bwd_w'))"
}
for spec in $KNOBS; do
  tag=${spec%%:*}; envs=${spec#*:}
  run $tag ${envs//,/ } || exit 1
done
