#!/bin/bash
# Debug: one streamed-projection test under several environments, short limits.
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for E in "KCTC_STREAM_DBG=0"; do
  i=$((i+1))
  env $E timeout -k 10 60 python -u -m pytest tests -m gpu -x -q --timeout 25 --timeout-method thread -k "streamed_gemms_match_unstreamed and KCTC_FWD_STREAM and 97" > gpurun_out/dbg2_$i.log 2>&1
  rc=$?
  echo "$E rc=$rc"; grep -E "passed|failed|Timeout|Error|assert" gpurun_out/dbg2_$i.log | head -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
