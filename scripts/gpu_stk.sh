#!/bin/bash
# stacked hi/lo MFMA operands (kPrecX3S): RNN / pinning / train / full-size
# parity, then bench with and without
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rnn_gpu.py tests/test_xcd_pin_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py > gpurun_out/stk_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout|rel" gpurun_out/stk_tests.log | head -30; tail -5 gpurun_out/stk_tests.log; exit 1; }
tail -2 gpurun_out/stk_tests.log
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/stk$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/stk$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/stk$tag.log').read().strip().splitlines()[-1]);lm=d['loss_match'];print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], lm['pass'], lm['max_rel_cost'], lm['logits_sketch_err'], lm['grad_sketch_err'])"
}
bench on KCTC_STK=1 && bench off KCTC_STK=0  # (STK default off)
