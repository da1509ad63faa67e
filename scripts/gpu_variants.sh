#!/bin/bash
# Bench variants of knobs: scripts/gpu_variants.sh "<test env>" name1 "ENV=.. ENV=.." name2 "..." ...
# First runs the recurrence/train GPU tests under <test env> (skip with "-"), then one
# short bench per variant, printing frames/s and the recurrence families.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TENV=$1; shift
if [ "$TENV" != "-" ]; then
  env $TENV timeout -k 10 300 python -u -m pytest tests/test_rnn_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/var_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/var_tests.log; exit 1; }
  tail -1 gpurun_out/var_tests.log
fi
while [ $# -ge 2 ]; do
  name=$1; envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-h2d-pass --steps 10 ${BENCH_ARGS:-} > gpurun_out/var_$name.log 2>&1 || { echo BENCH_FAILED $name; tail -20 gpurun_out/var_$name.log; exit 1; }
  python - "$name" gpurun_out/var_$name.log <<'PY'
import json,sys
j=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
f=j["roofline"]["families_ms_per_step"]
print(sys.argv[1], j["value"], "fwd", f.get("rnn_fwd_rec"), "bwd", f.get("rnn_bwd_rec"), "gw", f.get("gemm_bwd_w"), "gr", f.get("gemm_bwd_r"))
PY
done
