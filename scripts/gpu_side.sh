#!/bin/bash
# side-stream weight-GEMM block count A/B (KCTC_SIDE_BLOCKS)
set -o pipefail
mkdir -p gpurun_out
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d-pass > gpurun_out/sb$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/sb$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sb$tag.log').read().strip().splitlines()[-1]);f=d['roofline']['families_ms_per_step'];print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], d['loss_match']['pass'], f.get('clip_gradient'), f.get('gemm_bwd_w'), f.get('gemm_bwd_r'))"
}
bench def KCTC_X=0 && bench s256 KCTC_SIDE_BLOCKS=256 && bench s128 KCTC_SIDE_BLOCKS=128 && bench s64 KCTC_SIDE_BLOCKS=64
