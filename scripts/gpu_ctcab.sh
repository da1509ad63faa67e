#!/bin/bash
# CTC alpha/beta: parity tests, then the kernel timing probe (lagged offsets vs per-frame max)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "ctc or train_step or fullsize or decode or smoke" > gpurun_out/ctcab_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ctcab_tests.log; exit 1; }
tail -1 gpurun_out/ctcab_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctcl0 -o run --output-format csv -- python3 scripts/ctc_probe.py > gpurun_out/ctcl0.log 2>&1 || { echo PROBE0_FAILED; exit 1; }
KCTC_CTC_DBG=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctcl2 -o run --output-format csv -- python3 scripts/ctc_probe.py > gpurun_out/ctcl2.log 2>&1 || { echo PROBE2_FAILED; exit 1; }
grep -h alpha gpurun_out/ctcl0/run_kernel_stats.csv gpurun_out/ctcl2/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3
