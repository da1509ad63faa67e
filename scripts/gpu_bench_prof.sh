#!/bin/bash
# Round measurement: smoke, full default bench (with CPU baseline), rocprofv3
# kernel-trace/stats of the same workload, then two PMC passes (FETCH_SIZE,
# WRITE_SIZE; counters only with --kernel-trace) for the dominant kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-loss-match > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-loss-match > gpurun_out/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-loss-match > gpurun_out/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -20 gpurun_out/pmc_write.log; exit 1; }
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write rnn_bwd_rec gpurun_out/pmc_rnn_bwd_rec.json
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write rnn_fwd_rec gpurun_out/pmc_rnn_fwd_rec.json
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ctc_alpha_beta gpurun_out/pmc_ctc_alpha_beta.json
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ctc_grad gpurun_out/pmc_ctc_grad.json
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write ctc_logz gpurun_out/pmc_ctc_logz.json
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gemm_p256_kernel gpurun_out/pmc_gemm_p256.json
find gpurun_out/prof -name "*stats*"
