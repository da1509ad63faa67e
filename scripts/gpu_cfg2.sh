#!/bin/bash
# configs[2] bench (5xBLSTM-512, fs=3: T_max=667, N=64) + full-size parity printout
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/fullsize.log 2>&1 || { echo FULLSIZE_FAILED; tail -30 gpurun_out/fullsize.log; exit 1; }
grep -E "lstm512|rnn0|PASS|passed" gpurun_out/fullsize.log | cut -c1-400
timeout -k 10 600 python bench.py --config 2 --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_cfg2.log; exit 1; }
tail -1 gpurun_out/bench_cfg2.log
