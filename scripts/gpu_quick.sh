#!/bin/bash
# whole GPU suite, then a default bench and a trace of one step
set -o pipefail
mkdir -p gpurun_out/tr0
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/qb.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/qb.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/qb.log').read().strip().splitlines()[-1]);lm=d['loss_match'];print(d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], lm['pass'], lm['grad_sketch_err'])"
KCTC_REC_TRACE=gpurun_out/tr0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr0.log 2>&1 || { echo TRACE0_FAILED; tail -5 gpurun_out/tr0.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr0/rec_fwd.bin gpurun_out/tr0/rec_bwd.bin
