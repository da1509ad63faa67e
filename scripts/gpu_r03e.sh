#!/bin/bash
# Splice contexts (new tests + the egs / model-io / train suites they touch),
# then the configs[2] / configs[4] benches with rocprof stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_splice_gpu.py tests/test_train_egs_gpu.py tests/test_model_io_gpu.py tests/test_decode_gpu.py tests/test_egs.py > gpurun_out/r03e_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED" gpurun_out/r03e_tests.log | head -30; tail -5 gpurun_out/r03e_tests.log; exit 1; }
tail -2 gpurun_out/r03e_tests.log
bash scripts/gpu_cfg_prof.sh
