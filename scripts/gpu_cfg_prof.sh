#!/bin/bash
# measurement of configs[2] and configs[4]: bench (loss match), rocprofv3
# stats; configs[4] also PMC traffic and MFMA-utilisation passes
set -o pipefail
mkdir -p gpurun_out/keep
export TMPDIR=/tmp
for c in 2 4; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > gpurun_out/keep/cfg${c}_bench.log 2>&1 || { echo BENCH_FAILED $c; tail -5 gpurun_out/keep/cfg${c}_bench.log; exit 1; }
  tail -1 gpurun_out/keep/cfg${c}_bench.log | cut -c1-300
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-loss-match --no-h2d-pass > gpurun_out/prof_cfg$c.log 2>&1 || { echo PROF_FAILED $c; tail -5 gpurun_out/prof_cfg$c.log; exit 1; }
  find gpurun_out/prof_cfg$c -name "*kernel_stats*" -exec cp {} gpurun_out/keep/cfg${c}_kernel_stats.csv \;
  f=$(find gpurun_out/prof_cfg$c -name "*kernel_trace.csv" | head -1)
  python scripts/timeline.py $f 50 > gpurun_out/keep/cfg${c}_timeline.txt 2>&1 || true
  rm -rf gpurun_out/prof_cfg$c
done
B="python3 bench.py --config 4 --no-cpu-baseline --no-loss-match --no-h2d-pass --steps 1 --warmup 1 --no-profile"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -5 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -5 gpurun_out/pmc_write.log; exit 1; }
python - <<'PY'
import json, subprocess
out = {}
for k in ["rnn_bwd_rec", "rnn_fwd_rec", "gemm_p256_kernel", "x3p_splitk_reduce", "ctc_alpha_beta", "fillBufferAligned"]:
    subprocess.run(["python3", "scripts/pmc_traffic.py", "gpurun_out/pmc_fetch", "gpurun_out/pmc_write", k, "/tmp/t.json"],
                   check=False, capture_output=True)
    try:
        out[k] = json.load(open("/tmp/t.json"))
    except Exception as e:
        out[k] = {"error": str(e)}
json.dump(out, open("gpurun_out/keep/cfg4_pmc_traffic.json", "w"), indent=1)
print({k: v.get("traffic_bytes_per_launch") for k, v in out.items()})
PY
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_mfma -o run --output-format csv -- $B > gpurun_out/pmc_mfma.log 2>&1 || { echo PMC_MFMA_FAILED; tail -5 gpurun_out/pmc_mfma.log; exit 1; }
python3 scripts/pmc_mfma.py gpurun_out/pmc_mfma gpurun_out/keep/cfg4_pmc_mfma.json 256 rnn_fwd_rec=rnn_fwd_rec6@128 rnn_bwd_rec=rnn_bwd_rec6@128 gemm_p256_bf16=gemm_p256_kernel\<true gemm_p256_pair=gemm_p256_pair_kernel > /dev/null
rm -rf gpurun_out/pmc_mfma
ls gpurun_out/keep
