#!/bin/bash
# round-end check at HEAD: whole GPU suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['loss_match']['pass'], d['roofline']['frac'])"
