#!/bin/bash
# aggregated epochs for the streamed GEMMs of pinned recurrences: tests, then
# bench A/B over the streamed GEMMs' block counts
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xcd_pin_gpu.py tests/test_rnn_gpu.py > gpurun_out/agg_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/agg_tests.log | head -30; tail -5 gpurun_out/agg_tests.log; exit 1; }
tail -1 gpurun_out/agg_tests.log
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/agg$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/agg$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/agg$tag.log').read().strip().splitlines()[-1]);lm=d['loss_match'];f=d['roofline']['families_ms_per_step'];print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], lm['pass'], f['rnn_fwd_rec'], f['rnn_bwd_rec'])"
}
bench def KCTC_X=0 && bench f240 KCTC_STREAM_BLOCKS=240 && bench b240 KCTC_BWD_STREAM_BLOCKS=240 && bench f240b240 KCTC_STREAM_BLOCKS=240 KCTC_BWD_STREAM_BLOCKS=240 && bench nofs KCTC_FWD_STREAM=0
