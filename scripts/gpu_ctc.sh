#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_train_gpu.py tests/test_train_egs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_ctc.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests_ctc.log; exit 1; }
tail -2 gpurun_out/tests_ctc.log
bash scripts/gpu_sweep_nt.sh "KCTC_X=1"
python -c "import json; d=json.loads(open('gpurun_out/sweep_v1.log').read().strip().splitlines()[-1]); print({k:v for k,v in d['roofline']['families_ms_per_step'].items() if 'ctc' in k})"
