#!/bin/bash
# whole GPU suite (unless NO_SUITE), then one bench line per BASELINE config (loss match included)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NO_SUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
for c in ${CFGS:-1 2 4}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_cfg$c.log 2>&1 || { echo BENCH_FAILED $c; tail -5 gpurun_out/bench_cfg$c.log; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/bench_cfg$c.log").read().strip().splitlines()[-1])
r = d["roofline"]
print("cfg$c", d["value"], d["ms_per_step"], "h2d", (d.get("h2d_inclusive") or {}).get("value"), r["kernel"], r["frac"],
      r["secondary"].get("recurrence_step_us"), "loss_match", d["loss_match"] and d["loss_match"]["pass"])
PY
done
