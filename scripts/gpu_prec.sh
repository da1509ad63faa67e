#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for cfg in "KCTC_X=1" "KCTC_GEMM=f32 KCTC_FWD_REC=4 KCTC_BWD_REC=4"; do
  echo "== $cfg"; env $cfg timeout -k 10 300 python -u scripts/prec_train256.py 2>&1 | grep -v amdgpu.ids
done
