#!/bin/bash
# XCD-pinned backward as the default: CU-mask -> XCD map, bit-identity and
# CU-budget tests, RNN/train suites, bench with / without pinning.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/cumask_probe > gpurun_out/cumask.log 2>&1 && cat gpurun_out/cumask.log &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xcd_pin_gpu.py tests/test_cu_budget_gpu.py tests/test_rnn_gpu.py tests/test_train_gpu.py > gpurun_out/xprod_tests.log 2>&1 &&
tail -3 gpurun_out/xprod_tests.log &&
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/xb$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/xb$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/xb$tag.log').read().strip().splitlines()[-1]);print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
}
bench on KCTC_XCD6=1 && bench off KCTC_XCD6=0
