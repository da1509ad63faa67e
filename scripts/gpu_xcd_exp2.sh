#!/bin/bash
# XCD-local backward + partial-dh ring: per-step times (no streamed dx GEMM).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  mkdir -p gpurun_out/x$tag
  env "$@" KCTC_BWD_STREAM=0 KCTC_REC_TRACE=gpurun_out/x$tag timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-h2d-pass > gpurun_out/x$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/x$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/x$tag.log').read().strip().splitlines()[-1]);print('$tag', '$*', d['value'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'])"
  python scripts/trace_rec.py gpurun_out/x$tag/rec_bwd.bin | grep -E "flags|loads|reduced|stored|published|period|handoff|local"
}
run b KCTC_XCD6=1 && run c KCTC_XCD6=1 KCTC_BWD_RING=2 && run d KCTC_XCD6=1 KCTC_BWD_RING=4 && run e KCTC_BWD_RING=2
