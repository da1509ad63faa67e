#!/usr/bin/env python3
"""CTC-train frames/sec on MI355X (BASELINE.json metric, configs[1]).

One step = one NnetCtcUpdater::ComputeForMinibatch with SGD
(kctc_nnet_train_step) of the recipe model 5 x BLSTM-512 (Splice ->
[CuDNNRecurrent -> ClipGradient(30)] x 5 -> Affine(41)) on a synthetic
minibatch of N=16 utterances, T_max=2000, 40-dim features (BASELINE.md §2
generator, seed 20161015 + 1000*rank + step), fp32.  Inputs are resident in
HBM when the timed region starts (a second pass with the H2D copy inside
every step is reported beside it).  frames = sum of real frames T_n.

Multi-GPU: one process per GPU; each rank trains its own N=16 shard and the
weight gradients are summed with RCCL (kctc_nnet_enable_dp), so per-GPU work
is fixed ("weak" scaling).  `--gpus N` with no WORLD_SIZE in the environment
starts the N rank processes itself (torchrun-style env, LOCAL_RANK = device)
before anything touches the GPU; under torch.distributed.run it is one rank.
`--dp-transport host` sums the gradients through gloo on the host instead
(kctc_nnet_enable_dp_host): ranks may then share a device, each on its own
CU-masked share of it (kctc_set_cu_partition) -- a rehearsal of the N-rank
path on a one-GPU box, not a throughput configuration.

Before the timed region the bench checks the loss: one train step of the
committed full-size fixture of the measured config (tests/golden/
sketch_step*.npz, fp64 oracle, same parameters and minibatch) must match at
1e-4 -- configs[4] (bf16 operands) at its error model's per-output bar
(tests/sketch_common.py) -- (`loss_match`).

Three timed passes of K steps each, all after the warm-up:
  1. `value`: HBM-resident features, no profiling events (the measurement
     contract: inputs resident when the timed region starts; the trainer's
     boundary takes device features);
  2. the same with per-family HIP events on the trainer's streams, from which
     the `roofline` of the dominant kernel is priced (events cost a little
     time, so this pass is never `value`);
  3. `h2d_inclusive`: the features copied from pinned host memory inside every
     step -- SURVEY §8d's timed region, which starts at the H2D copy --
     reported beside `value` (the PCIe-inclusive rate is never `value`).

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP
events on the trainer's stream over the timed region) and a CPU baseline
(the oracle's fp32 restatement, OpenMP, on utterances of the GPU run's own
first timed minibatch with the run's initial parameters; rank 0 at N=1 only).
"""
import argparse
import json
import os
import socket
import subprocess
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
LOSS_BAR = 1e-4            # north_star: loss / grads within 1e-4 relative

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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=1, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] to measure (1: the metric's config)")
    ap.add_argument("--T", type=int, default=0)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--hidden", type=int, default=0)
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--dp-transport", choices=("rccl", "host"), default="rccl",
                    help="N>1: gradient sum over RCCL (one GPU per rank) or gloo on the host "
                         "(ranks may share a GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-h2d-pass", action="store_true")
    ap.add_argument("--no-loss-match", action="store_true")
    ap.add_argument("--average-every", type=int, default=0,
                    help="N>1: the recipe's model averaging every K steps instead of the per-step "
                         "gradient all-reduce (kctc_nnet_set_dp_mode 1)")
    return ap.parse_args(argv)


# ---- rank launcher ------------------------------------------------------------
def rank_envs(n, port, base=None):
    """torch.distributed.run-style environments of n local ranks (one node)."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
        out.append(e)
    return out


def device_of(local_rank, local_world, ndev, transport):
    """(device, cu part, cu parts) of a local rank: one device per rank over
    RCCL; over the host transport ranks wrap around the devices and the ranks
    on one device split its CUs."""
    if transport == "rccl":
        if local_rank >= ndev:
            raise SystemExit(f"bench.py: rank {local_rank} needs GPU {local_rank} but {ndev} are visible "
                             "(RCCL: one GPU per rank; --dp-transport host lets ranks share a GPU)")
        return local_rank, 0, 1
    dev = local_rank % ndev
    nparts = len(range(dev, local_world, ndev))
    return dev, local_rank // ndev, nparts


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, script=None):
    """Start n rank processes of this script (fresh children: nothing here has
    touched the GPU) and wait for all of them; a failed rank stops the rest
    and its exit status is returned.  Rank 0 prints the JSON line (the ranks
    sum their totals among themselves)."""
    port = free_port()
    procs = [subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=e)
             for e in rank_envs(n, port)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in procs:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


# ---- work and byte models -------------------------------------------------------
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
    return f


def ctc_bytes(T_max, A, num_frames, label_lengths):
    """Algorithmic HBM bytes of one minibatch's CTC kernels (ctc.hip), per
    utterance n with T_n frames and S_n = 2 L_n + 1 extended labels:
      ctc_logz       reads the T_max*N*A activations, writes the normalised
                     log-probs (T_max*N*A) and the per-frame log-normaliser;
      ctc_alpha_beta the alpha block and the beta block each read the T_n
                     emission rows (A floats) and write their spilled column
                     (T_n*S_n floats) and fp64 frame offsets (T_n);
      ctc_grad       reads both spills, both offset vectors, the activations
                     and the normaliser, writes the gradient (padding rows too)."""
    T = np.asarray(num_frames, np.float64)
    S = 2.0 * np.asarray(label_lengths, np.float64) + 1.0
    N = T.size
    rows = float(T_max * N)
    return {"ctc_logz": rows * A * 4 * 2 + rows * 4,
            "ctc_alpha_beta": float(np.sum(2 * (4 * T * A + 4 * T * S + 8 * T))),
            "ctc_grad": float(np.sum(8 * T * S + 16 * T + 4 * T * A + 4 * T)) + rows * A * 4}


def _committed_pmc(kind, config):
    """Newest committed rocprofv3 PMC summary of `kind` ("traffic" or "mfma")
    for `config`: profiles/rNN*_pmc_<kind>.json for configs[1],
    profiles/rNN*_cfg<N>_pmc_<kind>.json otherwise (scripts/gpu_prof.sh
    and scripts/gpu_cfg_prof.sh on this workload).  bench.py cannot read
    counters itself."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{kind}.json")))
    tag = f"_cfg{config}_"
    files = [f for f in files if (tag in os.path.basename(f)) == (config != 1)]
    out = []
    for f in reversed(files):
        try:
            out.append((json.load(open(f)), os.path.basename(f)))
        except (OSError, ValueError):
            continue
    return out


def pmc_traffic(kernel, config=1):
    """HBM-side bytes per launch of `kernel` (FETCH_SIZE x2 + WRITE_SIZE, the
    guide's gfx950 correction); (None, None) when none is committed."""
    for d, name in _committed_pmc("traffic", config):
        if kernel in d and "traffic_bytes_per_launch" in d[kernel]:
            return d[kernel]["traffic_bytes_per_launch"], name
    return None, None


def pmc_mfma(config=1):
    """Counter-based MFMA utilisation per kernel family (SQ_VALU_MFMA_BUSY_CYCLES
    against GRBM_GUI_ACTIVE x the 4 SIMDs of every CU; scripts/pmc_mfma.py)."""
    for d, name in _committed_pmc("mfma", config):
        return {"source": name, **d}
    return None


# ---- checks and baselines ---------------------------------------------------------
def loss_match(k, dev, case="cfg1"):
    """One train step of the committed full-size fixture of `case` (tests/golden/
    sketch_step*.npz, generated by tests/golden/make_sketch.py with the fp64
    oracle): configs[1] / [2] / [4] at their shapes, the fixture's parameters and
    bench.py's first minibatch.  Reports the per-utterance cost error, the
    network output's and every applied gradient's sketch error (norm-wise
    relative, tests/sketch_common.py) and the best-path flips against the
    fp64 output, each with its bar: 1e-4, or for configs[4] (bf16 operands)
    the error model's tolerance of that output (sketch_common.bf16_tol)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import sketch_common as S
    s = S.STEPS[case]
    g = np.load(os.path.join(ROOT, "tests", "golden", s["file"] + ".npz"))
    T, N, D, H, A, R = s["T"], s["N"], s["D"], s["H"], s["A"], s["R"]
    bf16 = s.get("prec") == "bf16"
    tol = (lambda what, c=0: float(S.bf16_tol(S.step_stages(R, what, c)))) if bf16 else (lambda what, c=0: LOSS_BAR)
    rnn, Wa, ba = S.step_params(S.ProductLayout(k), case)
    feats, nf, fl, ll = S.step_inputs(k, case)
    net = k.Nnet(k.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=s["lr"],
                                 max_seq_length=T, rnn_mode=s["mode"]), seed=1, device=dev.index)
    if bf16:
        net.set_precision("bf16")
    rnn_idx = [1 + 2 * c for c in range(R)]
    aff_idx = 2 * R + 1
    for c, i in enumerate(rnn_idx):
        net.set_params(i, rnn[c])
    net.set_params(aff_idx, np.concatenate([Wa.ravel(), ba]))
    net.srand(0)
    objf, acc, wt = net.train_step(torch.from_numpy(feats).to(dev), T, N, nf, fl, ll)
    costs = net.last_costs(N)
    rc = np.abs(costs - g["costs"]) / np.abs(g["costs"])
    logits = net.last_output(T, N, A)
    table = {"costs": (float(rc.max()), tol("costs")),
             "tot_objf": (abs(objf - float(g["tot_objf"])) / abs(float(g["tot_objf"])), tol("costs"))}
    samp = {}  # sampled entries' max |diff| / rms against SAMP_FACTOR x the bar

    def put(key, e, bar):
        table[key] = (max(e["norm"], e["proj"]), bar)
        samp[key] = (e["samp"], S.SAMP_FACTOR * bar)
    put("logits", S.compare(logits, S.load(g, "logits"), 500, tol("logits")), tol("logits"))
    for c, i in enumerate(rnn_idx):
        put(f"grad_rnn{c}", S.compare(np.clip(net.get_grad(i).astype(np.float64), -5.0, 5.0), S.load(g, f"g{c}"),
                                      600 + c, tol("grad", c)), tol("grad", c))
    put("grad_affine", S.compare(net.get_grad(aff_idx).astype(np.float64), S.load(g, "gaff"), 700, tol("affine")),
        tol("affine"))
    ids = net.last_best_path(T, N)
    net.close()
    grads = [v[0] for key, v in table.items() if key.startswith("grad_")]
    out = {"fixture": f"tests/golden/{s['file']}.npz (fp64 oracle, {case} step, params pseed {s['pseed']}, "
                      f"minibatch seed {s['seed']})",
           "max_rel_cost": table["costs"][0], "tot_objf_rel": table["tot_objf"][0],
           "logits_sketch_err": table["logits"][0], "grad_sketch_err": max(grads),
           "best_path_flips": int(np.sum(ids != g["ids"])), "frames": int(ids.size),
           "objf_per_label": objf / wt,
           "bar": "bf16 error model per output (tests/sketch_common.bf16_tol)" if bf16 else LOSS_BAR,
           "errors_vs_bar": {key: {"err": float("%.3g" % v[0]), "bar": float("%.3g" % v[1])}
                             for key, v in table.items()},
           "sampled_entries_vs_bar": {key: {"err": float("%.3g" % v[0]), "bar": float("%.3g" % v[1])}
                                      for key, v in samp.items()}}
    out["pass"] = bool(all(v[0] < v[1] for v in list(table.values()) + list(samp.values())) and
                       wt == float(g["tot_weight"]))
    return out


def cpu_baseline(params0, batch, T, D, H, A, L, ratio=0.125, mode=2, Ns=4):
    """The oracle's fp32 restatement (warp-ctc-CPU-style CTC + blocked-GEMM
    LSTM/affine, OpenMP) on a bounded sample of the GPU run's own bytes: the
    first Ns utterances of its first timed minibatch, the run's initial
    parameters (about 8 s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    s = O.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = L, mode, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, 5e-4, 5e-4
    rnn_p, aff = params0
    ps = [p.copy() for p in rnn_p]
    Wa = np.ascontiguousarray(aff[:A * 2 * H].reshape(A, 2 * H))
    ba = aff[A * 2 * H:].copy()
    feats, nf, fl, ll = batch
    N = nf.size
    sub = np.ascontiguousarray(feats.reshape(T, N, D)[:, :Ns, :])
    nlab = int(np.sum(ll[:Ns]))
    t0 = time.time()
    O.train_step(s, ps, Wa, ba, sub, nf[:Ns], fl[:nlab], ll[:Ns])
    dt = time.time() - t0
    frames = int(nf[:Ns].sum())
    return {"value": float(frames / dt), "unit": "frames/s", "cores": int(O.lib().oracle_num_threads()),
            "kind": "port",
            "sample": f"one full train step ({L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H} fwd+CTC+bwd+SGD, fp32) on "
                      f"utterances 0..{Ns - 1} of the GPU run's first timed minibatch (T_max={T}, {frames} frames, "
                      f"the run's initial parameters) in {dt:.1f}s"}


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    cf = CONFIGS[args.config]

    import torch
    import torch.distributed as dist
    import __graft_entry__ as ge

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")  # rendezvous (+ host transport)
    device, part, nparts = device_of(local, local_world, max(1, torch.cuda.device_count()), args.dp_transport)
    k = ge.load_package()
    if nparts > 1:
        k.set_cu_partition(part, nparts)
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    T, N, H = args.T or cf["T"], args.N or cf["N"], args.hidden or cf["H"]
    D, A, L, mode, ratio = 40, 41, args.layers, cf["mode"], cf["ratio"]
    nw = 4 if mode == 2 else 3
    cfg = k.recipe_config(num_rnn=L, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                          max_seq_length=T, rnn_mode=mode)
    net = k.Nnet(cfg, seed=20161015, device=device)  # same init on every rank
    bf16 = cf.get("prec") == "bf16"
    if bf16:
        net.set_precision("bf16")
    rnn_idx = [1 + 2 * c for c in range(L)]
    params0 = ([net.get_params(i) for i in rnn_idx], net.get_params(2 * L + 1))
    dp_info = None
    if world > 1:
        if args.average_every > 0:
            net.set_dp_mode("average")
        if args.dp_transport == "rccl":
            uid = k.dp_unique_id() if rank == 0 else bytes(128)
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            net.enable_dp(obj[0], rank, world)
        else:
            def allreduce(buf):
                dist.all_reduce(torch.from_numpy(buf))
            net.enable_dp_host(allreduce, world)
        dp_info = {"transport": args.dp_transport, "ranks": world,
                   "devices": len({device_of(r, local_world, max(1, torch.cuda.device_count()),
                                             args.dp_transport)[0] for r in range(local_world)}),
                   "ranks_per_device_cu_share": f"1/{nparts}" if nparts > 1 else "all",
                   "mode": "model averaging every %d steps" % args.average_every if args.average_every > 0
                   else "gradient sum every step"}

    lm = None

    total = args.warmup + args.steps
    batches, host_batches = [], []
    for step in range(total):
        feats, nf, fl, ll = k.synth_minibatch(20161015 + 1000 * rank + step, T, N, D, A, ratio)
        batches.append((torch.from_numpy(feats).to(dev), nf, fl, ll, torch.from_numpy(feats).pin_memory()))
        host_batches.append((feats, nf, fl, ll) if step == args.warmup else None)
    torch.cuda.synchronize()

    warm_stats = []
    for step in range(args.warmup):
        f, nf, fl, ll, _ = batches[step]
        warm_stats.append(net.train_step(f, T, N, nf, fl, ll))

    profile = not args.no_profile
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

    net.set_profiling(False)
    dt, frames, stats, step_ms = timed_pass(False)
    traj = np.array([[o, w] for o, _, w in warm_stats + stats], np.float64)
    objf = sum(o for o, _, _ in stats)
    acc = sum(a for _, a, _ in stats)
    wt = sum(w for _, _, w in stats)
    if world > 1:  # the loss / accuracy / label totals summed over the ranks
        tot = torch.tensor([objf, acc, wt], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        objf, acc, wt = float(tot[0]), float(tot[1]), float(tot[2])
        tt = torch.from_numpy(np.ascontiguousarray(traj))
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        traj = tt.numpy()
    fam_flops = model_flops(T, N, D, H, A, L, nw=nw)
    prof = {}
    prof_dt = None
    if profile:
        net.set_profiling(True)
        prof_dt, prof_frames, _, _ = timed_pass(False)
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
        if h2d:
            t2 = torch.tensor([h2d[0], float(h2d[1])], dtype=torch.float64)
            mx2 = t2.clone()
            dist.all_reduce(mx2, op=dist.ReduceOp.MAX)
            dist.all_reduce(t2, op=dist.ReduceOp.SUM)
            h2d = (float(mx2[0]), int(t2[1]), h2d[2])

    # the split-fp16 ("x3") products deliver fp32-class results on the f16
    # matrix cores: priced against the fp32 MFMA peak (the precision class,
    # the contract's `peak` for dtype f32) and against the engine they issue on
    peak_mfma = PEAK_F16_TFLOPS if bf16 else PEAK_FP32_TFLOPS
    peak_engine = PEAK_F16_TFLOPS if bf16 else PEAK_X3_TFLOPS
    engine = "bf16 MFMA (dense 2.5 PF)" if bf16 else "split-fp16 x3 on the f16 MFMA (2.5 PF / 3)"
    roof = None
    if prof:
        # the dominant KERNEL of the step's critical path: the GEMM families
        # on the trainer's compute stream run the packed GEMM kernel
        # (gemm_p256 / gemm_x3p) and are priced together against each
        # recurrence kernel; the weight-gradient GEMMs (gemm_bwd_w / _r) run on
        # the side stream BESIDE the next backward recurrence -- their spans
        # include the time they wait for CUs, so they are priced on their own
        # in `secondary.gate_gemm`, not picked as the dominant kernel
        kernels = {"rnn_fwd_rec": ["rnn_fwd_rec"], "rnn_bwd_rec": ["rnn_bwd_rec"],
                   "gemm_p256 (compute-stream gate GEMMs: fwd_proj, bwd_data)": ["gemm_fwd_proj", "gemm_bwd_data"]}
        # a family some of whose layers ran as a streamed GEMM (its own span
        # family) has fewer launches than layers: count that share of its FLOPs
        per_step = {"gemm_fwd_proj": L, "gemm_bwd_data": L - 1, "gemm_bwd_w": L, "gemm_bwd_r": L,
                    "rnn_fwd_rec": L, "rnn_bwd_rec": L}

        def fam_share(f):
            return min(1.0, prof[f][1] / args.steps / max(per_step[f], 1))
        ktime = {kn: (sum(prof[f][0] for f in fams if f in prof), sum(prof[f][1] for f in fams if f in prof),
                      sum(fam_flops[f] * fam_share(f) for f in fams if f in prof) * args.steps)
                 for kn, fams in kernels.items()}
        dom = max((kn for kn in ktime if ktime[kn][1]), key=lambda kn: ktime[kn][0])
        ms, n, flops_total = ktime[dom]
        avg_s = ms / n / 1e3
        flops_per_launch = flops_total / n
        achieved = flops_per_launch / avg_s / 1e12
        traffic, tsrc = pmc_traffic(dom, args.config)
        # a split-fp16 GEMM can outrun the fp32 MFMA peak (it issues on the f16
        # engine): then the engine it issues on is the peak (frac <= 1)
        peak = peak_mfma if achieved <= peak_mfma else peak_engine
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
                "peak_basis": ("bf16 dense MFMA peak (the dtype's)" if bf16 else
                               "fp32 MFMA peak (the precision class)" if peak == peak_mfma else
                               f"the engine the products issue on ({engine}); "
                               f"{achieved / peak_mfma:.2f}x the fp32 MFMA peak"),
                "kernel": dom, "avg_launch_ms": round(ms / n, 4), "flops_per_launch": flops_per_launch,
                "engine": {"name": engine, "peak": round(peak_engine, 1),
                           "frac": round(achieved / peak_engine, 4)},
                "families_ms_per_step": {f: round(prof[f][0] / args.steps, 3) for f in prof},
                "families_launches_per_step": {f: round(prof[f][1] / args.steps, 2) for f in prof}}
        aux = {}
        # the recurrences are serial over T: their step latency is the figure
        # that bounds them
        aux["recurrence_step_us"] = {f: round(prof[f][0] / prof[f][1] / T * 1e3, 3)
                                     for f in ("rnn_fwd_rec", "rnn_bwd_rec") if f in prof}
        # the input projections and dx GEMMs of layers 2..L stream off the
        # recurrences (no kernel time of their own to price); the weight-gradient
        # GEMM dW = dGates^T [x | 1] is the same packed kernel, timed on its own
        # (side stream, sharing the chip with a backward recurrence)
        if "gemm_bwd_w" in prof:
            ms_g, n_g = prof["gemm_bwd_w"]
            tf = fam_flops["gemm_bwd_w"] * args.steps / (ms_g / 1e3) / 1e12
            aux["gate_gemm"] = {"bound": "mfma",
                                "kernel": "gemm_bwd_w (gemm_x3p, %s)" % ("bf16" if bf16 else "split-fp16"),
                                "achieved": round(tf, 2), "peak": round(peak_engine, 1),
                                "unit": "TFLOP/s" if bf16 else "TFLOP/s (fp32-class)",
                                "frac": round(tf / peak_engine, 4), "where": "in step, beside a recurrence"}
            if rank == 0:
                # the same kernel on the same shape, alone on the chip
                G4, din = nw * H, 2 * H
                Ms, Ns, Ks = G4, din, T * N
                split = 4 if bf16 else 8
                ms_s = k.lib().kcm_bench_gemm_packed(None, Ms, Ns, Ks, 1 if bf16 else 0, 5, split)
                if ms_s > 0:
                    tf_s = 2.0 * Ms * Ns * Ks / (ms_s / 1e3) / 1e12
                    aux["gate_gemm"]["standalone"] = {
                        "shape": f"M={Ms} N={Ns} K={Ks} split-K {split} (dW of a BLSTM layer, one direction)",
                        "ms": round(ms_s, 4), "achieved": round(tf_s, 2), "frac": round(tf_s / peak_engine, 4),
                        "note": "kcm_bench_gemm_packed: random packed operands, 5 launches after 2 warm-ups"}
        # CTC: each kernel against its own algorithmic bytes
        cb = {"ctc_logz": 0.0, "ctc_alpha_beta": 0.0, "ctc_grad": 0.0}
        for step in range(args.warmup, total):
            _, nf, _, ll, _ = batches[step]
            for key, v in ctc_bytes(T, A, nf, ll).items():
                cb[key] += v
        for key, byts in cb.items():
            if key in prof:
                ms_c, n_c = prof[key]
                gbs = byts / (ms_c / 1e3) / 1e9
                aux[key] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": round(gbs / PEAK_HBM_GBS, 4), "ms_per_launch": round(ms_c / n_c, 4),
                            "bytes_per_launch": round(byts / n_c)}
        if "ctc_alpha_beta" in aux:
            aux["ctc_alpha_beta"]["us_per_frame"] = round(aux["ctc_alpha_beta"]["ms_per_launch"] / T * 1e3, 4)
            aux["ctc_alpha_beta"]["note"] = ("serial over T (one barrier per group of 8 frames): latency-bound; "
                                             "bytes = emission rows read + alpha/beta spill + fp64 offsets written")
        # counter evidence beside the algorithmic fractions (north_star's
        # "MFMA utilisation against gfx950 peak"): SQ_VALU_MFMA_BUSY_CYCLES
        # of each kernel family from the committed rocprofv3 pass
        aux["mfma_util_pmc"] = pmc_mfma(args.config)
        if prof_dt:
            aux["profiled_pass"] = {"value": round(prof_frames / prof_dt, 1),
                                    "note": "the same K steps with per-family HIP events (the roofline's "
                                            "source); not `value`"}
        roof["secondary"] = aux

    # after the timed passes: with this second Nnet created and freed before
    # them, the trainer's recurrences ran 2-4 % slower (configs[1]: 727.8k vs
    # 752.2k frames/s, same box, profiles/r05e_lossmatch_ab.txt)
    if rank == 0 and not args.no_loss_match and (T, N, H, L) == (cf["T"], cf["N"], cf["H"], 5):
        lm = loss_match(k, dev, {1: "cfg1", 2: "cfg2", 4: "cfg4"}[args.config])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(params0, host_batches[args.warmup], T, D, H, A, L, ratio, mode=mode,
                           Ns=2 if H > 512 else 4)

    if rank == 0:
        value = frames / dt
        fpf = step_flops_per_frame(D, H, A, L, nw=nw)
        step_tf = value * fpf / 1e12
        out = {"metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if bf16 else "f32",
               "data": f"synthetic (BASELINE.md generator: N(0,1) 40-dim features, T_n=T_max-floor(u*0.1*T_max), "
                       f"L_n=floor(T_n*{ratio}) labels in [1,40]); random-init weights (recipe init)",
               "config": {"workload": cf["name"] if (T, N, H) == (cf["T"], cf["N"], cf["H"]) else
                          f"custom: {L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H}, minibatch={N}/GPU, T_max={T}",
                          "model": f"{L}x{'BLSTM' if mode == 2 else 'BGRU'}-{H}+affine-{A}", "global_batch": N * world,
                          "seq_len": T, "parallelism": f"dp{world}"},
               "loss_match": lm,
               # per-step device time (HIP events on the trainer's stream): the
               # median of the K steps beside the whole-job mean
               "median_step_ms": round(med_ms, 3),
               "value_median": round(frames_per_step / (med_ms / 1e3), 1),
               # whole train step: algorithmic FLOPs/frame x frames/s against the
               # engine the products run on; the fp32 MFMA peak beside it as a
               # ratio (the x3 engine is faster than fp32 MFMA, so it may pass 1)
               "step_roofline": {"flops_per_frame": fpf, "achieved_tflops": round(step_tf, 2),
                                 "engine": engine, "peak": round(peak_engine, 1),
                                 "frac": round(step_tf / peak_engine, 4),
                                 "ratio_to_fp32_mfma_peak": None if bf16 else round(step_tf / PEAK_FP32_TFLOPS, 4)},
               "loss": {"objf_per_label": round(objf / max(wt, 1), 4), "accuracy": round(acc / max(wt, 1), 4),
                        # warm-up + timed steps in order (summed over the ranks);
                        # the growth is the reference's own SGD on this synthetic
                        # data: summed minibatch gradients at lr 5e-4 (tests/
                        # test_train_gpu.py::test_multistep_trajectory_matches_oracle)
                        "objf_per_label_by_step": [round(o / max(w, 1), 3) for o, w in traj]},
               "dp": dp_info, "roofline": roof, "cpu_baseline": cpu}
        if h2d:
            out["h2d_inclusive"] = {"value": round(h2d[1] / h2d[0], 1),
                                    "median_step_ms": round(float(np.median(h2d[2])), 3),
                                    "note": "features copied from pinned host memory on the trainer's stream "
                                            "inside every step (not `value`)"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
