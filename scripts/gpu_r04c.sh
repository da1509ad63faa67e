#!/bin/bash
# backward IO waves: traces and step times; then the gated projection probes
# (stream-ordered diagnostics first, the concurrent mode last)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
TRACES="base:X=0 iow:KCTC_BWD_IOW=1" $T 300 bash scripts/gpu_trace_diag.sh || exit 1
DIAGS="base:X=0 iow:KCTC_BWD_IOW=1 base2:X=0 iow2:KCTC_BWD_IOW=1" $T 400 bash scripts/gpu_diag.sh || exit 1
$T 120 python -u scripts/gate_probe.py off d1 d2 > gpurun_out/gate_probe1.log 2>&1; rc=$?; cat gpurun_out/gate_probe1.log | tail -5; [ $rc -eq 0 ] || exit 1
$T 60 python -u scripts/gate_probe.py off full > gpurun_out/gate_probe2.log 2>&1; rc=$?; cat gpurun_out/gate_probe2.log | tail -5; exit $rc
