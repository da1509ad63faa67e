#!/bin/bash
# round 5: backward variants A/B (stacked transposed vs plain, tagged vs flagged), parity, phase trace
set -o pipefail
mkdir -p gpurun_out/tr_b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_xcd_pin_gpu.py tests/test_fullsize_gpu.py tests/test_rnn_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/r05b_tests.log | head -30; tail -5 gpurun_out/r05b_tests.log; exit 1; }
tail -1 gpurun_out/r05b_tests.log
ab() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/ab_$tag.log 2>&1 || { echo "AB_FAILED $tag"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);r=d['roofline'];lm=d['loss_match']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], r['avg_launch_ms'], lm['pass'], lm['grad_sketch_err'])"
}
ab all_tag KCTC_STK_BWD=1 || exit 1
ab fwdflag KCTC_STK_BWD=1 KCTC_FWD_DTAG=0 || exit 1
ab bwdplain KCTC_STK_BWD=0 || exit 1
ab allflag KCTC_STK_BWD=1 KCTC_BWD_DTAG=0 KCTC_FWD_DTAG=0 || exit 1
ab all_tag2 KCTC_STK_BWD=1 || exit 1
ab bwdplain2 KCTC_STK_BWD=0 || exit 1
KCTC_REC_TRACE=gpurun_out/tr_b timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr_b.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr_b.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr_b/rec_bwd.bin gpurun_out/tr_b/rec_fwd.bin
rm -rf gpurun_out/tr_b
