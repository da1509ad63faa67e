#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
KCTC_FWD_STREAM=0 timeout -k 10 20 python -u scripts/stream_probe.py 30 4 256 > gpurun_out/probe$i.log 2>&1; rc=$?; echo "rc$i=$rc"; tail -14 gpurun_out/probe$i.log
[ $rc -eq 0 ] || exit 1
done
