#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/cumask_probe > gpurun_out/cumask.log 2>&1 && tail -4 gpurun_out/cumask.log &&
run() {  # tag args -- env...
  local tag=$1; shift
  local args=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass $args > gpurun_out/xd$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc args=[$args] env=[$*]"
  if [ $rc -eq 0 ]; then
    python -c "import json;d=json.loads(open('gpurun_out/xd$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
  else
    grep -E "Error|error" gpurun_out/xd$tag.log | tail -2
  fi
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run a "" && run b "" KCTC_XCD6=0 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xcd_pin_gpu.py tests/test_fullsize_gpu.py > gpurun_out/xprod_tests.log 2>&1; tail -3 gpurun_out/xprod_tests.log
