#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tr9
KCTC_FWD_SYNC=0 timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_f7.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_f7.log; exit 1; }
tail -2 gpurun_out/tests_f7.log
KCTC_FWD_SYNC=0 KCTC_REC_TRACE=gpurun_out/tr9 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/tr9.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/tr9.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr9/rec_fwd.bin
bash scripts/gpu_sweep_nt.sh "KCTC_FWD_SYNC=0" "KCTC_FWD_SYNC=0 KCTC_FWD_U=8" "KCTC_FWD_SYNC=1"
