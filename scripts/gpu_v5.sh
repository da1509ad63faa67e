#!/bin/bash
# v5 backward validation: parity tests, trace, bench variants.
set -o pipefail
mkdir -p gpurun_out/tr5
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_egs.py tests/test_train_egs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_v5.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_v5.log; exit 1; }
tail -2 gpurun_out/tests_v5.log
KCTC_BWD_U=8 timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_v5u8.log 2>&1 || { echo TESTS_U8_FAILED; tail -40 gpurun_out/tests_v5u8.log; exit 1; }
tail -1 gpurun_out/tests_v5u8.log
KCTC_REC_TRACE=gpurun_out/tr5 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr5.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr5.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr5/rec_bwd.bin
for cfg in "KCTC_BWD_REC=5" "KCTC_BWD_U=8" "KCTC_BWD_REC=4"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { echo BENCH_FAILED $cfg; tail -5 gpurun_out/bench_$cfg.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg |', d['value'], d['ms_per_step'], d['roofline']['families_ms_per_step'])"
done
