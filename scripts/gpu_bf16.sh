#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -k "bf16 or row_groups" -v -s --timeout 240 --timeout-method thread > gpurun_out/bf16.log 2>&1; rc=$?
grep -E "^\(|PASS|FAIL|Error|passed|failed|^[0-9] " gpurun_out/bf16.log | cut -c1-300
exit $rc
