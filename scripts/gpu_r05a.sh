#!/bin/bash
# round 5: self-tagged backward hand-off -- parity of the pinned recurrences, A/B bench, phase trace
set -o pipefail
mkdir -p gpurun_out/tr_tag gpurun_out/tr_flag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_xcd_pin_gpu.py tests/test_fullsize_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/r05a_tests.log | head -30; tail -5 gpurun_out/r05a_tests.log; exit 1; }
tail -1 gpurun_out/r05a_tests.log
ab() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/ab_$tag.log 2>&1 || { echo "AB_FAILED $tag"; tail -3 gpurun_out/ab_$tag.log; return 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]);r=d['roofline'];lm=d['loss_match']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], r['avg_launch_ms'], lm['pass'], lm['grad_sketch_err'])"
}
ab tag KCTC_BWD_DTAG=1 || exit 1
ab flag KCTC_BWD_DTAG=0 || exit 1
ab tag2 KCTC_BWD_DTAG=1 || exit 1
KCTC_REC_TRACE=gpurun_out/tr_tag timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr_tag.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr_tag.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr_tag/rec_bwd.bin
KCTC_BWD_DTAG=0 KCTC_REC_TRACE=gpurun_out/tr_flag timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr_flag.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr_flag.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr_flag/rec_bwd.bin
