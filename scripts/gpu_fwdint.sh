#!/bin/bash
# what slows the forward recurrence beside its streamed projection:
# timing diagnostics (KCTC_DIAG_NOPF: 1 skips the next-step input loads, 2 the
# row-major output stores -- wrong results, timing only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bench() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-h2d-pass --no-loss-match > gpurun_out/fi$tag.log 2>&1 || { echo ${tag}_FAILED; tail -5 gpurun_out/fi$tag.log; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/fi$tag.log').read().strip().splitlines()[-1]);f=d['roofline']['families_ms_per_step'];print('$tag', '$*', d['value'], d['ms_per_step'], d['roofline']['secondary']['recurrence_step_us'], f['rnn_fwd_rec'], f.get('fwd_proj_stream'))"
}
bench def KCTC_X=0 && bench nopf1 KCTC_DIAG_NOPF=1 && bench nopf2 KCTC_DIAG_NOPF=2 && bench nopf3 KCTC_DIAG_NOPF=3 && bench nofs KCTC_FWD_STREAM=0 && bench nofs_nopf3 KCTC_FWD_STREAM=0 KCTC_DIAG_NOPF=3 && bench sb64 KCTC_STREAM_BLOCKS=128
