#!/bin/bash
# parity of the backward recurrence's direct consumer, then bench (with recurrence step times)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_xcd_pin_gpu.py tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py tests/test_component_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/dir_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/dir_tests.log | head -30; tail -40 gpurun_out/dir_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/dir_tests.log | tail -1
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/dir_bench.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/dir_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/dir_bench.log').read().strip().splitlines()[-1]);r=d['roofline'];lm=d['loss_match']
print(d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], lm['pass'], lm['grad_sketch_err'], lm['max_rel_cost'])"
