#!/bin/bash
# recurrence phase traces (KCTC_REC_TRACE) under diagnostic settings: TRACES="tag:ENV=V,ENV2=V ..."
set -o pipefail
mkdir -p gpurun_out
for spec in $TRACES; do
  tag=${spec%%:*}; envs=${spec#*:}
  mkdir -p gpurun_out/tr_$tag
  env ${envs//,/ } KCTC_REC_TRACE=gpurun_out/tr_$tag timeout -k 10 200 python bench.py --config ${CFG:-1} --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tr_$tag.log 2>&1 || { echo TRACE_FAILED $tag; tail -3 gpurun_out/tr_$tag.log; exit 1; }
  echo "== $tag"; python scripts/trace_rec.py gpurun_out/tr_$tag/rec_fwd.bin gpurun_out/tr_$tag/rec_bwd.bin | grep -v "shader clock" | tee gpurun_out/tr_$tag.txt
  rm -f gpurun_out/tr_$tag/*.bin  # (the stamps are tens of MB; the summary stays)
done
