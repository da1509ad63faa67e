#!/bin/bash
# One selected GPU test under a short time limit (debugging).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -k "$1" > gpurun_out/dbg_tests.log 2>&1
rc=$?
tail -60 gpurun_out/dbg_tests.log
exit $rc
