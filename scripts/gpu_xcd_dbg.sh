#!/bin/bash
# Pinned backward + streamed dx GEMM timing out in the bench: which variant.
# A variant exiting 1 (a Python error) lets the next run; anything else stops.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag args -- env...
  local tag=$1; shift
  local args=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-h2d-pass --no-loss-match $args > gpurun_out/xd$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc args=[$args] env=[$*]"
  if [ $rc -eq 0 ]; then
    python -c "import json;d=json.loads(open('gpurun_out/xd$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'])"
  else
    grep -E "Error|error" gpurun_out/xd$tag.log | tail -2
  fi
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run a "" && run b "--no-profile" && run c "" KCTC_BWD_STREAM_BLOCKS=96 && run d "" KCTC_BWD_STREAM=0 &&
mkdir -p gpurun_out/xdtr && run e "" KCTC_REC_TRACE=gpurun_out/xdtr
ls gpurun_out/xdtr 2>/dev/null
