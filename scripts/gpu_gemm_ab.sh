#!/bin/bash
# A/B of the 256-tile packed GEMM k loop (KCTC_P256=1: DMA block per stage,
# 2: DMA spread over the MFMAs) on the train step's shapes, then the GEMM /
# RNN / train-step parity tests on the new default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2 1 2; do
  echo "== KCTC_P256=$v" >> gpurun_out/gemm_ab.log
  KCTC_P256=$v timeout -k 10 120 python scripts/gemm_packed_bench.py >> gpurun_out/gemm_ab.log 2>&1 || { echo GEMM_BENCH_FAILED; tail -20 gpurun_out/gemm_ab.log; exit 1; }
done
cat gpurun_out/gemm_ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_cumatrix_gpu.py > gpurun_out/gemm_ab_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gemm_ab_tests.log; exit 1; }
tail -3 gpurun_out/gemm_ab_tests.log
