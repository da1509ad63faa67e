#!/bin/bash
# v6 forward validation: RNN parity tests, full train-step tests, trace, bench.
set -o pipefail
mkdir -p gpurun_out/tr8
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_train_egs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_f6.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_f6.log; exit 1; }
tail -2 gpurun_out/tests_f6.log
KCTC_FWD_U=16 KCTC_BWD_U=8 timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_f6u.log 2>&1 || { echo TESTS_U_FAILED; tail -40 gpurun_out/tests_f6u.log; exit 1; }
tail -1 gpurun_out/tests_f6u.log
KCTC_REC_TRACE=gpurun_out/tr8 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr8.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr8.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr8/rec_fwd.bin
bash scripts/gpu_sweep_nt.sh "KCTC_FWD_REC=6" "KCTC_FWD_U=16" "KCTC_FWD_REC=4"
