#!/usr/bin/env python3
"""CTC-train frames/sec on MI355X (BASELINE.json metric, configs[1]).

One step = one NnetCtcUpdater::ComputeForMinibatch with SGD
(kctc_nnet_train_step) of the recipe model 5 x BLSTM-512 (Splice ->
[CuDNNRecurrent -> ClipGradient(30)] x 5 -> Affine(41)) on a synthetic
minibatch of N=16 utterances, T_max=2000, 40-dim features (BASELINE.md §2
generator, seed 20161015 + 1000*rank + step), fp32.  Inputs are uploaded to
HBM before the timed region.  frames = sum of real frames T_n.

Multi-GPU: one process per GPU (torch.distributed.run); each rank trains its
own N=16 shard, weight gradients are summed with RCCL (kctc_nnet_enable_dp),
so per-GPU work is fixed ("weak" scaling).

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP
events on the trainer's stream over the timed region) and a CPU baseline
(the oracle's fp32 restatement, OpenMP, bounded sample; rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CTC-train frames/sec, 5×BLSTM-512 mb=16, at 1/2/4/8 MI355X; loss match"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix = FP32 vector peak (dense)
PEAK_HBM_GBS = 8000.0
PEAK_F16_TFLOPS = 2500.0   # dense f16/bf16 MFMA


def model_flops(T, N, D, H, A, L, nw=4, dirs=2):
    """Algorithmic FLOPs per launch family for one step (all L layers)."""
    TN = T * N
    f = {}
    din = [D] + [dirs * H] * (L - 1)
    f["gemm_fwd_proj"] = sum(2.0 * TN * nw * H * dirs * d for d in din)
    f["rnn_fwd_rec"] = L * 2.0 * TN * nw * H * H * dirs
    f["rnn_bwd_rec"] = L * 2.0 * TN * nw * H * H * dirs
    f["gemm_bwd_data"] = sum(2.0 * TN * nw * H * dirs * d for d in din[1:])  # layer 1 dx not needed
    f["gemm_bwd_w"] = sum(2.0 * TN * nw * H * dirs * d for d in din)
    f["gemm_bwd_r"] = L * 2.0 * (T - 1) * N * nw * H * H * dirs
    launches = {"gemm_fwd_proj": L, "rnn_fwd_rec": L, "rnn_bwd_rec": L, "gemm_bwd_data": 2 * (L - 1),
                "gemm_bwd_w": L, "gemm_bwd_r": L}
    return f, launches


def pmc_traffic(kernel):
    """HBM-side bytes per launch of `kernel` from the newest committed rocprofv3
    PMC pass (profiles/*_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE; produced by
    scripts/gpu_bench_prof.sh on this workload).  bench.py cannot read counters
    itself; None when no measurement of this kernel is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d and "traffic_bytes_per_launch" in d[kernel]:
            return d[kernel]["traffic_bytes_per_launch"], os.path.basename(f)
    return None, None


def cpu_baseline(T, D, H, A, L, steps_seed):
    """The oracle's fp32 restatement (warp-ctc-CPU-style CTC + blocked-GEMM
    LSTM/affine, OpenMP) on a bounded sample: 6 utterances of the same shape."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import __graft_entry__ as ge
    k = ge.load_package()
    Ns = 6
    s = O.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = L, 2, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, 5e-4, 5e-4
    rng = np.random.default_rng(0)
    ps = [(rng.standard_normal(O.params_size(2, D if i == 0 else 2 * H, H, 1, 2)) * 0.02).astype(np.float32)
          for i in range(L)]
    Wa = (rng.standard_normal((A, 2 * H)) / np.sqrt(2 * H)).astype(np.float32)
    ba = rng.standard_normal(A).astype(np.float32)
    feats, nf, fl, ll = k.synth_minibatch(steps_seed, T, Ns, D, A, 0.125)
    t0 = time.time()
    O.train_step(s, ps, Wa, ba, feats.reshape(T, Ns, D), nf, fl, ll)
    dt = time.time() - t0
    return {"value": float(nf.sum() / dt), "unit": "frames/s", "cores": int(O.lib().oracle_num_threads()),
            "kind": "port",
            "sample": f"one full train step (5xBLSTM-512 fwd+CTC+bwd+SGD, fp32) on {Ns} utterances "
                      f"x T_max={T} ({int(nf.sum())} frames) in {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--T", type=int, default=2000)
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import __graft_entry__ as ge

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")  # rendezvous only; data path is RCCL
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    k = ge.load_package()
    T, N, D, H, A, L = args.T, args.N, 40, args.hidden, 41, args.layers
    cfg = k.recipe_config(num_rnn=L, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                          max_seq_length=T)
    net = k.Nnet(cfg, seed=20161015, device=local)  # same init on every rank
    if world > 1:
        uid = k.dp_unique_id() if rank == 0 else bytes(128)
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        net.enable_dp(obj[0], rank, world)

    total = args.warmup + args.steps
    batches = []
    for step in range(total):
        feats, nf, fl, ll = k.synth_minibatch(20161015 + 1000 * rank + step, T, N, D, A, 0.125)
        batches.append((torch.from_numpy(feats).to(dev), nf, fl, ll))
    torch.cuda.synchronize()

    for step in range(args.warmup):
        f, nf, fl, ll = batches[step]
        net.train_step(f, T, N, nf, fl, ll)

    profile = not args.no_profile
    net.set_profiling(profile)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    frames = 0
    objf = wt = acc = 0.0
    # pipelined host loop: each call queues a step and returns the stats of
    # the step before the previous one; the flush (inside the timed region)
    # waits for the rest
    stats = []
    for step in range(args.warmup, total):
        f, nf, fl, ll = batches[step]
        r = net.train_step_async(f, T, N, nf, fl, ll)
        if r is not None:
            stats.append(r)
        frames += int(nf.sum())
    stats += net.train_flush()
    barrier()
    assert len(stats) == total - args.warmup
    for o, a, w in stats:
        objf, acc, wt = objf + o, acc + a, wt + w
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt, float(frames)], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        dt, frames = float(mx[0]), int(sm[1])

    fam_flops, _ = model_flops(T, N, D, H, A, L)
    prof = {}
    if profile:
        # *_stream / x3_pack_chain / x3_pack_bwd_stream: GEMMs and packs on the
        # overlap streams, running concurrently with the recurrence that feeds
        # them (their spans include the waiting); off the critical path
        for fam in list(fam_flops) + ["x3_pack", "x3_pack_w", "ctc_logz", "ctc_alpha_beta", "ctc_grad", "affine",
                                      "clip_gradient", "update", "argmax", "scale", "fwd_proj_stream",
                                      "bwd_data_stream", "x3_pack_chain", "x3_pack_bwd_stream"]:
            ms, n = net.profile(fam)
            if n:
                prof[fam] = (ms, n)
    roof = None
    if prof:
        dom = max((f for f in prof if f in fam_flops), key=lambda f: prof[f][0])
        ms, n = prof[dom]
        avg_s = ms / n / 1e3
        flops_per_launch = fam_flops[dom] / (n / args.steps)
        achieved = flops_per_launch / avg_s / 1e12
        traffic, tsrc = pmc_traffic(dom)
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel": dom,
                "avg_launch_ms": round(ms / n, 4),
                "flops_per_launch": flops_per_launch,
                "families_ms_per_step": {f: round(prof[f][0] / args.steps, 3) for f in prof}}
        # secondary rooflines named by north_star: the gate GEMMs (input
        # projections; split-fp16 MFMA: 3 f16 MFMAs per fp32-class product, so
        # the matrix-core issue rate is 3x the algorithmic rate against the
        # 2.5 PF dense f16 peak) and the CTC alpha/beta recursion (HBM bytes:
        # gathered emissions read + alpha/beta columns spilled, fp64 offsets)
        aux = {}
        # the input projections and dx GEMMs of layers 2..L now stream off the
        # recurrences (no kernel time of their own to price); the weight-gradient
        # GEMM dW = dGates^T [x | 1] is the same packed split-fp16 kernel, timed
        # on its own (side stream, not hidden behind anything it waits for)
        if "gemm_bwd_w" in prof:
            ms_g, n_g = prof["gemm_bwd_w"]
            tf = fam_flops["gemm_bwd_w"] * args.steps / (ms_g / 1e3) / 1e12
            aux["gate_gemm"] = {"bound": "mfma", "kernel": "gemm_bwd_w (gemm_x3p)", "achieved": round(tf, 2),
                                "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / PEAK_FP32_TFLOPS, 4),
                                "mfma_issue_frac_f16": round(3 * tf / PEAK_F16_TFLOPS, 4)}
        if "ctc_alpha_beta" in prof:
            ms_c, n_c = prof["ctc_alpha_beta"]
            byts = 0.0
            for step in range(args.warmup, total):
                _, nf, fl, ll = batches[step]
                S = 2 * np.asarray(ll, np.float64) + 1
                byts += float(np.sum(2 * (8.0 * np.asarray(nf) * S + 8.0 * np.asarray(nf))))
            gbs = byts / (ms_c / 1e3) / 1e9
            aux["ctc_alpha_beta"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                                     "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                                     "ms_per_launch": round(ms_c / n_c, 4),
                                     "note": "serial over T (one barrier per frame): latency-bound"}
        roof["secondary"] = aux

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(T, D, H, A, L, 20161015)

    if rank == 0:
        value = frames / dt
        out = {"metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (BASELINE.md generator: N(0,1) 40-dim features, T_n=T_max-floor(u*0.1*T_max), "
                       "L_n=floor(T_n/8) labels in [1,40]); random-init weights (recipe init)",
               "config": {"workload": f"configs[1]: librispeech CTC-monophone {L}xBLSTM-{H}, fs=1, "
                                      f"minibatch={N}/GPU, T_max={T}, fp32",
                          "model": f"{L}xBLSTM-{H}+affine-{A}", "global_batch": N * world, "seq_len": T,
                          "parallelism": f"dp{world}"},
               "loss": {"objf_per_label": round(objf / max(wt, 1), 4), "accuracy": round(acc / max(wt, 1), 4)},
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
