#!/bin/bash
# probe (3 small steps), streamed-GEMM parity tests, bench variants
set -o pipefail
bash scripts/gpu_probe.sh || exit 1
bash scripts/gpu_stream.sh "$@"
