#!/bin/bash
# forward IO waves: parity tests, then bench A/B (IO waves on / off, streamed projection on / off)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rnn_gpu.py tests/test_xcd_pin_gpu.py tests/test_train_gpu.py > gpurun_out/iow_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/iow_tests.log | head -30; tail -5 gpurun_out/iow_tests.log; exit 1; }
tail -1 gpurun_out/iow_tests.log
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/iow$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/iow$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/iow$tag.log').read().strip().splitlines()[-1]);lm=d['loss_match'];f=d['roofline']['families_ms_per_step'];print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], lm['pass'], lm['grad_sketch_err'], f['rnn_fwd_rec'], f.get('fwd_proj_stream'))"
}
bench iow KCTC_FWD_IOW=1 && bench noiow KCTC_FWD_IOW=0 && bench iow_nofs KCTC_FWD_IOW=1 KCTC_FWD_STREAM=0
