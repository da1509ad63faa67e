#!/bin/bash
# XCD-pinned forward: bit-identity tests (fwd + bwd pinning), RNN / train
# suites, then the bench with the forward pinned and not.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xcd_pin_gpu.py > gpurun_out/xf_pin.log 2>&1 || { echo PIN_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/xf_pin.log | head -30; tail -5 gpurun_out/xf_pin.log; exit 1; }
tail -2 gpurun_out/xf_pin.log
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/xf$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/xf$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/xf$tag.log').read().strip().splitlines()[-1]);print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
}
bench fon KCTC_XCD6F=1 && bench foff KCTC_XCD6F=0 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py tests/test_cu_budget_gpu.py > gpurun_out/xf_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/xf_tests.log | head -30; tail -5 gpurun_out/xf_tests.log; exit 1; }
tail -2 gpurun_out/xf_tests.log
