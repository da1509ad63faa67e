#!/bin/bash
# Row groups of 8 sequences (KCTC_REC_GS=8): parity tests, then the configs[1]
# bench with 16-row groups (default) and with 8-row groups.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "group8" > gpurun_out/gs8_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gs8_tests.log; exit 1; }
tail -2 gpurun_out/gs8_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_gs16.log 2>&1 || { echo BENCH16_FAILED; tail -20 gpurun_out/bench_gs16.log; exit 1; }
tail -1 gpurun_out/bench_gs16.log | cut -c1-400
KCTC_REC_GS=8 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_gs8.log 2>&1 || { echo BENCH8_FAILED; tail -20 gpurun_out/bench_gs8.log; exit 1; }
tail -1 gpurun_out/bench_gs8.log | cut -c1-400
