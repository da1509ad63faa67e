#!/bin/bash
# CTC alpha/beta in groups of m frames per barrier: parity tests at m = 2, 3, 4,
# then the timing probe for m = 1..4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 8 2; do
  KCTC_CTC_PAIR=$m timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "ctc or train_step_full or cfg0 or train_steps_match" > gpurun_out/ctcpair_tests_$m.log 2>&1 || { echo TESTS_FAILED m=$m; tail -40 gpurun_out/ctcpair_tests_$m.log; exit 1; }
  echo "m=$m $(tail -1 gpurun_out/ctcpair_tests_$m.log)"
done
for m in 1 8; do
  KCTC_CTC_PAIR=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ctcm$m -o run --output-format csv -- python3 scripts/ctc_probe.py > gpurun_out/ctcm$m.log 2>&1 || { echo PROBE_FAILED $m; exit 1; }
  echo "m=$m $(grep -h alpha gpurun_out/ctcm$m/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f3 | tr '\n' ' ')"
done
