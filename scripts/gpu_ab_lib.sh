#!/bin/bash
# same-box A/B of library builds: LIBS="base new" copies ab/<tag>.so over
# kaldi-ctc_amd/libkaldictc_amd.so and runs, ${ROUNDS:-2} times interleaved,
# either bench.py on configs[${CFG:-1}] or $CMD (its output printed as is)
set -o pipefail
mkdir -p gpurun_out
LIB=kaldi-ctc_amd/libkaldictc_amd.so
cp $LIB gpurun_out/.lib_keep.so
restore() { cp gpurun_out/.lib_keep.so $LIB; rm -f gpurun_out/.lib_keep.so; }
for round in $(seq ${ROUNDS:-2}); do
  for tag in $LIBS; do
    cp ab/$tag.so $LIB
    log=gpurun_out/ab_${tag}_$round.log
    if [ -n "$CMD" ]; then
      timeout -k 10 300 $CMD > $log 2>&1 || { echo "FAILED $tag"; tail -3 $log; restore; exit 1; }
      grep -v amdgpu.ids $log | sed "s/^/$tag: /"
      continue
    fi
    timeout -k 10 300 python bench.py --config ${CFG:-1} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-loss-match --no-h2d-pass > $log 2>&1 || { echo "FAILED $tag"; tail -3 $log; restore; exit 1; }
    python -c "
import json;d=json.loads(open('$log').read().strip().splitlines()[-1]);r=d['roofline']
print('$tag', d['value'], d['ms_per_step'], r['secondary']['recurrence_step_us'], {k:v for k,v in r['families_ms_per_step'].items() if k in ('bwd_data_stream','fwd_proj_rows','rnn_bwd_rec','rnn_fwd_rec')})"
  done
done
restore
