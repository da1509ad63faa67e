#!/bin/bash
# parity tests, then a recurrence trace and bench variants
set -o pipefail
mkdir -p gpurun_out/trq
timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_rnn_gpu.py tests/test_train_gpu.py tests/test_train_egs_gpu.py -q -k "not 256" --timeout 120 --timeout-method thread > gpurun_out/tests_q.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_q.log; exit 1; }
tail -2 gpurun_out/tests_q.log
KCTC_REC_TRACE=gpurun_out/trq timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/trq.log 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/trq.log; exit 1; }
python scripts/trace_rec.py gpurun_out/trq/rec_fwd.bin gpurun_out/trq/rec_bwd.bin
bash scripts/gpu_sweep_nt.sh "$@"
python -c "import json; d=json.loads(open('gpurun_out/sweep_v1.log').read().strip().splitlines()[-1]); print(d['roofline']['families_ms_per_step'])"
