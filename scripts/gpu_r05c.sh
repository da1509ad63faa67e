#!/bin/bash
# round 5: parity of the changed paths, then bench + timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_xcd_pin_gpu.py tests/test_fullsize_gpu.py tests/test_train_gpu.py tests/test_component_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/r05c_tests.log | head -30; tail -5 gpurun_out/r05c_tests.log; exit 1; }
tail -1 gpurun_out/r05c_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/r05c_bench.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r05c_bench.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05c_bench.log').read().strip().splitlines()[-1]);r=d['roofline'];lm=d['loss_match']
print(d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], r['kernel'], r['frac'], lm['pass'], lm['grad_sketch_err'])"
bash scripts/gpu_r05_tl.sh | tail -40
