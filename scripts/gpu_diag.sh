#!/bin/bash
# recurrence step times under diagnostic knobs (wrong results where noted), one bench per setting
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config ${CFG:-1} --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-loss-match --no-h2d-pass > gpurun_out/diag_$tag.log 2>&1 || { echo "DIAG_FAILED $tag"; tail -3 gpurun_out/diag_$tag.log; return 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/diag_$tag.log').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'])"
}
for spec in $DIAGS; do
  tag=${spec%%:*}; envs=${spec#*:}
  run $tag ${envs//,/ } || exit 1
done
