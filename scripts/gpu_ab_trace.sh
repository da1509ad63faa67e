#!/bin/bash
# phase traces of the configs[2] forward recurrence: current vs r03f recurrence source
set -o pipefail
mkdir -p gpurun_out/trn gpurun_out/tro
cp kaldi-ctc_amd/libkaldictc_amd.so gpurun_out/keep.so
KCTC_REC_TRACE=gpurun_out/trn timeout -k 10 300 python bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/trn.log 2>&1 &&
python scripts/trace_rec.py gpurun_out/trn/rec_fwd.bin &&
cp kaldi-ctc_amd/lib_r03f_rnn.so kaldi-ctc_amd/libkaldictc_amd.so &&
KCTC_REC_TRACE=gpurun_out/tro timeout -k 10 300 python bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-profile --no-loss-match --no-h2d-pass > gpurun_out/tro.log 2>&1 &&
python scripts/trace_rec.py gpurun_out/tro/rec_fwd.bin; rc=$?
cp gpurun_out/keep.so kaldi-ctc_amd/libkaldictc_amd.so; rm -f gpurun_out/keep.so
exit $rc
