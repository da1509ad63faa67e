#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for c in 2 4; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/c$c.log 2>&1 || { echo C${c}_FAILED; tail -5 gpurun_out/c$c.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c$c.log').read().strip().splitlines()[-1]);print($c, d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'])"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/c1.log 2>&1 || { echo C1_FAILED; tail -5 gpurun_out/c1.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c1.log').read().strip().splitlines()[-1]);print(1, d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
