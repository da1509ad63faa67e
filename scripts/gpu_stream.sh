#!/bin/bash
# streamed forward projection: parity tests, then bench with / without
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -v -k "stream or 256" --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/stream_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/stream_tests.log | tail -12
bash scripts/gpu_sweep_nt.sh "$@"
python -c "import json; d=json.loads(open('gpurun_out/sweep_v1.log').read().strip().splitlines()[-1]); print(d['roofline']['families_ms_per_step'])"
