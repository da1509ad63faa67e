#!/bin/bash
# CTC alpha/beta two frames per barrier: parity tests, then the timing probe (paired vs single frames)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "ctc or train_step or fullsize or decode or smoke or cfg0" > gpurun_out/ctcpair_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ctcpair_tests.log; exit 1; }
tail -1 gpurun_out/ctcpair_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctcq1 -o run --output-format csv -- python3 scripts/ctc_probe.py > gpurun_out/ctcq1.log 2>&1 || { echo PROBE1_FAILED; exit 1; }
KCTC_CTC_PAIR=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctcq0 -o run --output-format csv -- python3 scripts/ctc_probe.py > gpurun_out/ctcq0.log 2>&1 || { echo PROBE0_FAILED; exit 1; }
grep -h alpha gpurun_out/ctcq1/run_kernel_stats.csv gpurun_out/ctcq0/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3
