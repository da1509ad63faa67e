#!/usr/bin/env python3
"""CTC-train frames/sec on MI355X (BASELINE.json metric, configs[1]).

One step = one NnetCtcUpdater::ComputeForMinibatch with SGD
(kctc_nnet_train_step) of the recipe model 5 x BLSTM-512 (Splice ->
[CuDNNRecurrent -> ClipGradient(30)] x 5 -> Affine(41)) on a synthetic
minibatch of N=16 utterances, T_max=2000, 40-dim features (BASELINE.md §2
generator, seed 20161015 + 1000*rank + step), fp32.  Inputs are resident in
HBM when the timed region starts (a second pass with the H2D copy inside
every step is reported beside it).  frames = sum of real frames T_n.

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
# a split-fp16 ("x3") fp32-class product issues 3 f16 MFMAs: its ceiling on
# the engine it runs on is a third of the dense f16 peak
PEAK_X3_TFLOPS = PEAK_F16_TFLOPS / 3

# BASELINE.json configs this bench measures (--config): T_max, N/GPU, hidden,
# rnn mode, labels per frame (12.5 phones/s: 1/8 per 10-ms frame, 3/8 after
# frame_subsampling_factor 3), description
CONFIGS = {
    1: dict(T=2000, N=16, H=512, mode=2, ratio=0.125, fs=1,
            name="configs[1]: librispeech CTC-monophone 5xBLSTM-512, fs=1, minibatch=16/GPU, T_max=2000, fp32"),
    2: dict(T=667, N=64, H=512, mode=2, ratio=0.375, fs=3,
            name="configs[2]: librispeech CTC-monophone 5xBLSTM-512, fs=3 (google config), minibatch=64/GPU, "
                 "T_max=667, fp32"),
    4: dict(T=2000, N=32, H=1024, mode=3, ratio=0.125, fs=1, prec="bf16",
            name="configs[4]: 5xBGRU-1024, bf16 recurrences and MFMA gate GEMMs (fp32 accumulation, fp32 "
                 "master weights), minibatch=32/GPU, T_max=2000"),
}


def step_flops_per_frame(D, H, A, L, nw=4, dirs=2):
    """Algorithmic train-step FLOPs per frame (forward =
    sum_layers 2*dirs*nW*H*(D_in+H) + affine 2*2H*A; train = 3x forward)."""
    din = [D] + [dirs * H] * (L - 1)
    fwd = sum(2.0 * dirs * nw * H * (d + H) for d in din) + 2.0 * dirs * H * A
    return 3.0 * fwd


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


def cpu_baseline(T, D, H, A, L, steps_seed, ratio=0.125, mode=2, Ns=4):
    """The oracle's fp32 restatement (warp-ctc-CPU-style CTC + blocked-GEMM
    LSTM/affine, OpenMP) on a bounded sample: 4 utterances of the same shape
    (about 7 s of CPU work, so it does not dominate the bench's lease)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import __graft_entry__ as ge
    k = ge.load_package()
    s = O.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = L, mode, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, 5e-4, 5e-4
    rng = np.random.default_rng(0)
    ps = [(rng.standard_normal(O.params_size(mode, D if i == 0 else 2 * H, H, 1, 2)) * 0.02).astype(np.float32)
          for i in range(L)]
    Wa = (rng.standard_normal((A, 2 * H)) / np.sqrt(2 * H)).astype(np.float32)
    ba = rng.standard_normal(A).astype(np.float32)
    feats, nf, fl, ll = k.synth_minibatch(steps_seed, T, Ns, D, A, ratio)
    t0 = time.time()
    O.train_step(s, ps, Wa, ba, feats.reshape(T, Ns, D), nf, fl, ll)
    dt = time.time() - t0
    return {"value": float(nf.sum() / dt), "unit": "frames/s", "cores": int(O.lib().oracle_num_threads()),
            "kind": "port",
            "sample": f"one full train step ({L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H} fwd+CTC+bwd+SGD, fp32) on {Ns} utterances "
                      f"x T_max={T} ({int(nf.sum())} frames) in {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=1, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] to measure (1: the metric's config)")
    ap.add_argument("--T", type=int, default=0)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--hidden", type=int, default=0)
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-h2d-pass", action="store_true")
    ap.add_argument("--average-every", type=int, default=0,
                    help="N>1: the recipe's model averaging every K steps instead of the per-step "
                         "gradient all-reduce (kctc_nnet_set_dp_mode 1)")
    args = ap.parse_args()
    cf = CONFIGS[args.config]

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
    T, N, H = args.T or cf["T"], args.N or cf["N"], args.hidden or cf["H"]
    D, A, L, mode, ratio = 40, 41, args.layers, cf["mode"], cf["ratio"]
    nw = 4 if mode == 2 else 3
    cfg = k.recipe_config(num_rnn=L, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                          max_seq_length=T, rnn_mode=mode)
    net = k.Nnet(cfg, seed=20161015, device=local)  # same init on every rank
    bf16 = cf.get("prec") == "bf16"
    if bf16:
        net.set_precision("bf16")
    peak_mfma = PEAK_F16_TFLOPS if bf16 else PEAK_FP32_TFLOPS
    if world > 1:
        uid = k.dp_unique_id() if rank == 0 else bytes(128)
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        if args.average_every > 0:
            net.set_dp_mode("average")
        net.enable_dp(obj[0], rank, world)

    total = args.warmup + args.steps
    batches = []
    for step in range(total):
        feats, nf, fl, ll = k.synth_minibatch(20161015 + 1000 * rank + step, T, N, D, A, ratio)
        batches.append((torch.from_numpy(feats).to(dev), nf, fl, ll, torch.from_numpy(feats).pin_memory()))
    torch.cuda.synchronize()

    for step in range(args.warmup):
        f, nf, fl, ll, _ = batches[step]
        net.train_step(f, T, N, nf, fl, ll)

    profile = not args.no_profile
    net.set_profiling(profile)
    ext = torch.cuda.ExternalStream(net.stream, device=dev)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def timed_pass(h2d):
        """K steps, pipelined host loop (each call queues a step and returns
        the stats of the step before the previous one; the flush inside the
        timed region waits for the rest).  h2d: the features are copied from
        pinned host memory on the trainer's stream at the start of each step
        (SURVEY §8d's timed region); else they are resident in HBM.  HIP
        events on the trainer's stream mark every step's start."""
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        staging = [torch.empty_like(batches[0][0]) for _ in range(3)] if h2d else None
        barrier()
        t0 = time.perf_counter()
        frames, stats = 0, []
        for i, step in enumerate(range(args.warmup, total)):
            f, nf, fl, ll, fh = batches[step]
            evs[i].record(ext)
            if h2d:
                with torch.cuda.stream(ext):
                    f = staging[i % 3]
                    f.copy_(fh, non_blocking=True)
            r = net.train_step_async(f, T, N, nf, fl, ll)
            if r is not None:
                stats.append(r)
            frames += int(nf.sum())
            if world > 1 and args.average_every > 0 and (i + 1) % args.average_every == 0:
                stats += net.train_flush()
                net.average_params()
        stats += net.train_flush()
        evs[-1].record(ext)
        barrier()
        dt = time.perf_counter() - t0
        assert len(stats) == args.steps
        step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
        return dt, frames, stats, step_ms

    dt, frames, stats, step_ms = timed_pass(False)
    objf = sum(o for o, _, _ in stats)
    acc = sum(a for _, a, _ in stats)
    wt = sum(w for _, _, w in stats)
    if world > 1:  # the loss / accuracy / label totals summed over the ranks
        tot = torch.tensor([objf, acc, wt], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        objf, acc, wt = float(tot[0]), float(tot[1]), float(tot[2])
    fam_flops, _ = model_flops(T, N, D, H, A, L, nw=nw)
    if args.config != 1:
        # the committed PMC traffic was measured on configs[1]
        globals()["pmc_traffic"] = lambda kernel: (None, None)
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
    net.set_profiling(False)
    h2d = None
    if not args.no_h2d_pass:
        dt2, frames2, _, step_ms2 = timed_pass(True)
        h2d = (dt2, frames2, step_ms2)

    med_ms = float(np.median(step_ms))
    frames_per_step = frames / args.steps
    if world > 1:
        t = torch.tensor([dt, float(frames), med_ms], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        dt, frames, med_ms = float(mx[0]), int(sm[1]), float(mx[2])
        frames_per_step = frames / args.steps

    roof = None
    if prof:
        dom = max((f for f in prof if f in fam_flops), key=lambda f: prof[f][0])
        ms, n = prof[dom]
        avg_s = ms / n / 1e3
        flops_per_launch = fam_flops[dom] / (n / args.steps)
        achieved = flops_per_launch / avg_s / 1e12
        traffic, tsrc = pmc_traffic(dom)
        # the recurrences multiply on the split-fp16 (x3) path: priced against
        # the fp32 MFMA peak (the precision class they deliver) and, as
        # issue_frac, against what the f16 engine they run on could do
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak_mfma, "unit": "TFLOP/s",
                "frac": round(achieved / peak_mfma, 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel": dom,
                "avg_launch_ms": round(ms / n, 4),
                "flops_per_launch": flops_per_launch,
                "issue_frac_x3_on_f16": None if bf16 else round(achieved / PEAK_X3_TFLOPS, 4),
                "families_ms_per_step": {f: round(prof[f][0] / args.steps, 3) for f in prof}}
        aux = {}
        # the input projections and dx GEMMs of layers 2..L stream off the
        # recurrences (no kernel time of their own to price); the weight-gradient
        # GEMM dW = dGates^T [x | 1] is the same packed split-fp16 kernel, timed
        # on its own (side stream); its ceiling is the f16 engine / 3
        if "gemm_bwd_w" in prof and bf16:
            ms_g, n_g = prof["gemm_bwd_w"]
            tf = fam_flops["gemm_bwd_w"] * args.steps / (ms_g / 1e3) / 1e12
            aux["gate_gemm"] = {"bound": "mfma", "kernel": "gemm_bwd_w (gemm_x3p, bf16 operands)",
                                "achieved": round(tf, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                                "frac": round(tf / PEAK_F16_TFLOPS, 4)}
        elif "gemm_bwd_w" in prof:
            ms_g, n_g = prof["gemm_bwd_w"]
            tf = fam_flops["gemm_bwd_w"] * args.steps / (ms_g / 1e3) / 1e12
            aux["gate_gemm"] = {"bound": "mfma", "kernel": "gemm_bwd_w (gemm_x3p, split-fp16)", "achieved": round(tf, 2),
                                "peak": round(PEAK_X3_TFLOPS, 1), "unit": "TFLOP/s (fp32-class)",
                                "frac": round(tf / PEAK_X3_TFLOPS, 4),
                                "note": "peak = 2.5 PF dense f16 / 3 MFMAs per split-fp16 product; "
                                        "vs the fp32 MFMA peak it is " + str(round(tf / PEAK_FP32_TFLOPS, 3))}
        if "gate_gemm" in aux and rank == 0:
            # the same kernel on the same shape, alone on the chip (the in-step
            # figure above shares the CUs and memory system with a recurrence)
            G4, din = nw * H, 2 * H
            Ms, Ns, Ks = G4, din, T * N
            split = 4 if bf16 else 8
            ms_s = k.lib().kcm_bench_gemm_packed(None, Ms, Ns, Ks, 1 if bf16 else 0, 5, split)
            if ms_s > 0:
                tf_s = 2.0 * Ms * Ns * Ks / (ms_s / 1e3) / 1e12
                aux["gate_gemm"]["standalone"] = {
                    "shape": f"M={Ms} N={Ns} K={Ks} split-K {split} (dW of a BLSTM layer, one direction)",
                    "ms": round(ms_s, 4), "achieved": round(tf_s, 2),
                    "frac": round(tf_s / (PEAK_F16_TFLOPS if bf16 else PEAK_X3_TFLOPS), 4),
                    "mfma_issue_frac": round(tf_s * (1 if bf16 else 3) / PEAK_F16_TFLOPS, 4),
                    "note": "kcm_bench_gemm_packed: random packed operands, 5 launches after 2 warm-ups"}
        if "ctc_alpha_beta" in prof:
            ms_c, n_c = prof["ctc_alpha_beta"]
            byts = 0.0
            for step in range(args.warmup, total):
                _, nf, fl, ll, _ = batches[step]
                S = 2 * np.asarray(ll, np.float64) + 1
                byts += float(np.sum(2 * (8.0 * np.asarray(nf) * S + 8.0 * np.asarray(nf))))
            gbs = byts / (ms_c / 1e3) / 1e9
            aux["ctc_alpha_beta"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                                     "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                                     "ms_per_launch": round(ms_c / n_c, 4),
                                     "note": "serial over T (one barrier per group of 8 frames): latency-bound"}
        roof["secondary"] = aux

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(T, D, H, A, L, 20161015, ratio, mode=mode, Ns=2 if H > 512 else 4)

    if rank == 0:
        value = frames / dt
        fpf = step_flops_per_frame(D, H, A, L, nw=nw)
        out = {"metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if bf16 else "f32",
               "data": f"synthetic (BASELINE.md generator: N(0,1) 40-dim features, T_n=T_max-floor(u*0.1*T_max), "
                       f"L_n=floor(T_n*{ratio}) labels in [1,40]); random-init weights (recipe init)",
               "config": {"workload": cf["name"] if (T, N, H) == (cf["T"], cf["N"], cf["H"]) else
                          f"custom: {L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H}, minibatch={N}/GPU, T_max={T}",
                          "model": f"{L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H}+affine-{A}", "global_batch": N * world,
                          "seq_len": T, "parallelism": f"dp{world}"},
               # per-step device time (HIP events on the trainer's stream): the
               # median of the K steps beside the whole-job mean
               "median_step_ms": round(med_ms, 3),
               "value_median": round(frames_per_step / (med_ms / 1e3), 1),
               # whole train step against the fp32 MFMA peak (algorithmic
               # FLOPs/frame x frames/s; BASELINE.md's whole-step fraction)
               "step_roofline": {"flops_per_frame": fpf, "achieved_tflops": round(value * fpf / 1e12, 2),
                                 "peak": peak_mfma, "frac": round(value * fpf / 1e12 / peak_mfma, 4)},
               "loss": {"objf_per_label": round(objf / max(wt, 1), 4), "accuracy": round(acc / max(wt, 1), 4)},
               "roofline": roof, "cpu_baseline": cpu}
        if h2d:
            out["h2d_inclusive"] = {"value": round(h2d[1] / h2d[0], 1),
                                    "median_step_ms": round(float(np.median(h2d[2])), 3),
                                    "note": "features copied from pinned host memory on the trainer's stream "
                                            "inside every step (not `value`)"}
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
