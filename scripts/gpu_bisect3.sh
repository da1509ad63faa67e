#!/bin/bash
# bisect the configs[1] full-size cost mismatch across stream knobs
set -o pipefail
mkdir -p gpurun_out
T="tests/test_fullsize_gpu.py::test_train_step_full_size_matches_oracle[cfg1]"
for spec in tail0:KCTC_STREAM_TAIL=0 tail1:KCTC_STREAM_TAIL=1 rows0:KCTC_FWD_ROWS=0 base:X=1; do
  tag=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 200 python -u -m pytest "$T" -x -q -s --timeout 180 --timeout-method thread > gpurun_out/bis3_$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc $(grep -E 'passed|failed' gpurun_out/bis3_$tag.log | tail -1) $(grep -o 'max cost rel err.*' gpurun_out/bis3_$tag.log | head -1)"
  [ $rc -gt 1 ] && exit 1
done
exit 0
