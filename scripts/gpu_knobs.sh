#!/bin/bash
# env-knob A/B on the current tree: dx-stream blocks, poll sleep
set -o pipefail
mkdir -p gpurun_out
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/kn$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/kn$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/kn$tag.log').read().strip().splitlines()[-1]);print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
}
bench def KCTC_X=0 && bench bs224 KCTC_BWD_STREAM_BLOCKS=224 && bench bs160 KCTC_BWD_STREAM_BLOCKS=160 && bench ps0 KCTC_POLL_SLEEP=0 && bench def2 KCTC_X=0
