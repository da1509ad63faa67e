#!/bin/bash
# round measurement, configs[1]: smoke, default bench, rocprofv3 stats +
# timeline, PMC traffic (FETCH_SIZE / WRITE_SIZE) and MFMA-utilisation
# (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) passes, and the
# recurrence phase trace.  Large raw outputs are summarised and removed.
set -o pipefail
mkdir -p gpurun_out/keep
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-loss-match --no-h2d-pass"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/keep/bench_full.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/keep/bench_full.log; exit 1; }
tail -1 gpurun_out/keep/bench_full.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_bench.log; exit 1; }
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f 30 > gpurun_out/keep/timeline.txt 2>&1 || true
find gpurun_out/prof -name "*kernel_stats*" -exec cp {} gpurun_out/keep/kernel_stats.csv \;
rm -rf gpurun_out/prof
echo "stats + timeline done"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 1 --no-profile > gpurun_out/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -5 gpurun_out/pmc_fetch.log; exit 1; }
echo "FETCH_SIZE pass done"
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- $B --steps 1 --warmup 1 --no-profile > gpurun_out/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -5 gpurun_out/pmc_write.log; exit 1; }
echo "WRITE_SIZE pass done"
python - <<'PY'
import json, subprocess
out = {}
for k in ["rnn_bwd_rec", "rnn_fwd_rec", "ctc_alpha_beta", "ctc_grad", "ctc_logz", "gemm_p256_kernel",
          "gemm_p256_pair_kernel", "x3p_bwd_stream256_kernel<8", "x3p_bwd_stream256_kernel<4"]:
    subprocess.run(["python3", "scripts/pmc_traffic.py", "gpurun_out/pmc_fetch", "gpurun_out/pmc_write", k, "/tmp/t.json"],
                   check=False, capture_output=True)
    try:
        out[k] = json.load(open("/tmp/t.json"))
    except Exception as e:
        out[k] = {"error": str(e)}
json.dump(out, open("gpurun_out/keep/pmc_traffic.json", "w"), indent=1)
print({k: v.get("traffic_bytes_per_launch") for k, v in out.items()})
PY
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_mfma -o run --output-format csv -- $B --steps 1 --warmup 1 --no-profile > gpurun_out/pmc_mfma.log 2>&1 || { echo PMC_MFMA_FAILED; tail -5 gpurun_out/pmc_mfma.log; exit 1; }
python3 scripts/pmc_mfma.py gpurun_out/pmc_mfma gpurun_out/keep/pmc_mfma.json 256 rnn_fwd_rec=rnn_fwd_rec6@128 rnn_bwd_rec=rnn_bwd_rec6@128 gemm_p256=gemm_p256_kernel gemm_p256_pair=gemm_p256_pair_kernel dx_stream=x3p_bwd_stream256_kernel\<8 fwd_row_stream=x3p_bwd_stream256_kernel\<4 > /dev/null
rm -rf gpurun_out/pmc_mfma
echo "MFMA pass done"
TRACES="base:X=0" timeout -k 10 150 bash scripts/gpu_trace_diag.sh > gpurun_out/keep/trace_summary.txt 2>&1 || { echo TRACE_FAILED; tail -5 gpurun_out/keep/trace_summary.txt; exit 1; }
rm -rf gpurun_out/tr_base
ls gpurun_out/keep
