#!/bin/bash
# XCD-local recurrence experiment: parity with KCTC_XCD6=1, then bench variants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KCTC_XCD6=1 timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xcd_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/xcd_tests.log; exit 1; }
tail -1 gpurun_out/xcd_tests.log
run() { # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-h2d-pass --steps 10 > gpurun_out/xcd_$name.log 2>&1 || { echo BENCH_FAILED $name; tail -20 gpurun_out/xcd_$name.log; exit 1; }
  python - "$name" gpurun_out/xcd_$name.log <<'PY'
import json,sys
j=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
f=j["roofline"]["families_ms_per_step"]
print(sys.argv[1], j["value"], "fwd", f.get("rnn_fwd_rec"), "bwd", f.get("rnn_bwd_rec"))
PY
}
run base KCTC_X=0 || exit 1
run nostream KCTC_BWD_STREAM=0 || exit 1
run xcd_nostream KCTC_BWD_STREAM=0 KCTC_XCD6=1 || exit 1
