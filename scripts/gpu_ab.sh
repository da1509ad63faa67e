#!/bin/bash
# A/B of environment settings on configs[${CFG:-1}]: ABS="tag:ENV=V,ENV2=V tag2:..." (alternated twice);
# TESTS="tests/..." runs first (parity); TL=1 adds a timeline of the default build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest $TESTS -x -v -s --durations=15 --timeout ${PTIME:-120} --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/ab_tests.log | head -30; tail -60 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for rep in 1 2; do
  for spec in $ABS; do
    tag=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "-" ] && envs=""
    env ${envs//,/ } timeout -k 10 300 python bench.py --config ${CFG:-1} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-h2d-pass --no-profile > gpurun_out/ab_${tag}_$rep.log 2>&1; rc=$?
    # a KctcError (exit 1: the step's bounded waits timed out and drained) is reported and the A/B goes on; anything else ends the run
    if [ $rc -ne 0 ]; then echo "FAILED $tag rc=$rc: $(tail -1 gpurun_out/ab_${tag}_$rep.log | cut -c1-160)"; [ $rc -eq 1 ] && continue; exit 1; fi
    python -c "
import json;d=json.loads(open('gpurun_out/ab_${tag}_$rep.log').read().strip().splitlines()[-1]);lm=d.get('loss_match') or {}
print('$tag', $rep, d['value'], d['ms_per_step'], d.get('median_step_ms'), lm.get('pass'))"
  done
done
if [ -n "$TL" ]; then bash scripts/gpu_r05_tl.sh | tail -60; fi
