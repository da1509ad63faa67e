#!/bin/bash
# Selected GPU tests (pytest -k "$1"), then the configs[1] bench under each
# environment given as further arguments ("-" = default), summarised.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL="$1"; shift
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$SEL" > gpurun_out/sel_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/sel_tests.log; exit 1; }
  tail -1 gpurun_out/sel_tests.log
fi
i=0
for E in "$@"; do
  i=$((i+1))
  if [ "$E" = "-" ]; then E=""; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline $BARGS > gpurun_out/bench_$i.log 2>&1 || { echo BENCH_FAILED $E; tail -20 gpurun_out/bench_$i.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/bench_$i.log').read().strip().splitlines()[-1])
f=d['roofline']['families_ms_per_step']
print('$E', d['value'], d['ms_per_step'], {k:v for k,v in f.items() if v>0.3})"
done
