#!/bin/bash
# run a selection of GPU tests verbosely: scripts/gpu_sel.sh <pytest args...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/sel.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed|^[a-z0-9_]+ \{|^\{" gpurun_out/sel.log | cut -c1-400 | tail -60
exit $rc
