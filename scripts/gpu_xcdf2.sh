#!/bin/bash
# pinned recurrences after moving the write-through copies behind the hand-off
# loads: bit-identity + streamed-GEMM tests, bench, phase trace
set -o pipefail
mkdir -p gpurun_out/tr0
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xcd_pin_gpu.py tests/test_rnn_gpu.py > gpurun_out/xf_pin.log 2>&1 || { echo PIN_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/xf_pin.log | head -30; tail -5 gpurun_out/xf_pin.log; exit 1; }
tail -2 gpurun_out/xf_pin.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/xf_b.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/xf_b.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/xf_b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
KCTC_REC_TRACE=gpurun_out/tr0 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr0.log 2>&1 || { echo TRACE0_FAILED; tail -5 gpurun_out/tr0.log; exit 1; }
python scripts/trace_rec.py gpurun_out/tr0/rec_fwd.bin gpurun_out/tr0/rec_bwd.bin
