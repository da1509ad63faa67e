#!/bin/bash
# v6 backward validation: RNN parity tests, full train-step tests, trace, bench.
set -o pipefail
mkdir -p gpurun_out/tr7
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_v6.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_v6.log; exit 1; }
tail -2 gpurun_out/tests_v6.log
KCTC_BWD_U=8 timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_v6u8.log 2>&1 || { echo TESTS_U8_FAILED; tail -40 gpurun_out/tests_v6u8.log; exit 1; }
tail -1 gpurun_out/tests_v6u8.log
KCTC_REC_TRACE=gpurun_out/tr7 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr7.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr7.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr7/rec_bwd.bin
bash scripts/gpu_sweep_nt.sh "KCTC_BWD_REC=6" "KCTC_BWD_U=8" "KCTC_BWD_REC=4"
