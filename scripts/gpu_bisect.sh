#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
t() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u -m pytest "tests/test_fullsize_gpu.py::test_train_step_full_size_matches_oracle[cfg1]" -x -q --timeout 240 --timeout-method thread > gpurun_out/bis_$tag.log 2>&1; echo "$tag rc=$? $(tail -1 gpurun_out/bis_$tag.log)"; }
t blocks96 KCTC_BWD_STREAM_BLOCKS=192
t noprepack KCTC_PREPACK=0
t default X=0
