#!/bin/bash
# A/B on one box: current recurrence source vs the r03f one (lib_r03f_rnn.so), configs[2] / [4] / [1]
set -o pipefail
mkdir -p gpurun_out
cp kaldi-ctc_amd/libkaldictc_amd.so gpurun_out/keep.so
run() {  # tag config
  timeout -k 10 300 python bench.py --config $2 --steps 8 --warmup 2 --no-cpu-baseline --no-h2d-pass --no-loss-match > gpurun_out/ab$1_$2.log 2>&1 || { echo $1_$2_FAILED; tail -5 gpurun_out/ab$1_$2.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab$1_$2.log').read().strip().splitlines()[-1]);print('$1', $2, d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'])"
}
run new 2 && run new 4 && run new 1; rc=$?
cp gpurun_out/keep.so kaldi-ctc_amd/libkaldictc_amd.so; rm -f gpurun_out/keep.so
exit $rc
