#!/bin/bash
# bisect the pinned/unpinned mismatch: one test under several env settings
set -o pipefail
mkdir -p gpurun_out
T="tests/test_xcd_pin_gpu.py::test_pinned_bit_identical[2-16-400-KCTC_XCD6]"
for spec in base:X=1 pa0:KCTC_PACK_AVOID=0 s128:KCTC_BWD_S256=0 b48:KCTC_BWD_S256_BLOCKS=48 pair0:KCTC_WGRAD_PAIR=0; do
  tag=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 120 python -u -m pytest "$T" -x -q --timeout 100 --timeout-method thread > gpurun_out/bis_$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc $(grep -E 'passed|failed' gpurun_out/bis_$tag.log | tail -1) $(grep -o 'At index.*' gpurun_out/bis_$tag.log | head -1)"
  [ $rc -gt 1 ] && exit 1
done
exit 0
