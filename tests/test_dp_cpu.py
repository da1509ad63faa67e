"""Data-parallel semantics on CPU (world_size 2, gloo) -- the host logic of the
RCCL path (train_api.cpp RcclExchange): each rank back-propagates its own
utterance shard, the weight gradients are SUM-all-reduced, then the reference's
per-component update (RNN dW clipped to +-clip-gradient, W += lr * dW) runs on
every rank.  Checked against the fp64 oracle on the concatenated minibatch:
with the clip inactive the two are the same SGD step.

The oracle's train step updates in place; with lr = 1 and clip-gradient = inf
the parameter delta IS the summed gradient, which is what a rank contributes
to the all-reduce."""
import os

import numpy as np
import pytest


def _spec(oracle, R, H, D, A, clip=1e30, lr=1.0):
    s = oracle.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = R, 2, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 0.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = clip, lr, lr
    return s


def _params(oracle, R, H, D, A, seed=0):
    rng = np.random.default_rng(seed)
    ps = [rng.standard_normal(oracle.params_size(2, D if i == 0 else 2 * H, H, 1, 2)) * 0.2 for i in range(R)]
    Wa = rng.standard_normal((A, 2 * H)) / np.sqrt(2 * H)
    ba = rng.standard_normal(A)
    return ps, Wa, ba


def _shard_grads(oracle, feats, nf, fl, ll, R, H, D, A):
    ps, Wa, ba = _params(oracle, R, H, D, A)
    p0 = [p.copy() for p in ps] + [Wa.copy(), ba.copy()]
    T, N, _ = feats.shape
    tot, acc, wt = oracle.train_step(_spec(oracle, R, H, D, A), ps, Wa, ba, feats, nf, fl, ll)
    return [a - b for a, b in zip(ps + [Wa, ba], p0)], np.array([tot, acc, wt])


def _split(kctc, T, N, D, A, seed):
    feats, nf, fl, ll = kctc.synth_minibatch(seed, T, N, D, A, 0.2)
    f = feats.reshape(T, N, D).astype(np.float64)
    offs = np.concatenate([[0], np.cumsum(ll)])
    shards = []
    half = N // 2
    for lo, hi in ((0, half), (half, N)):
        sub_nf = nf[lo:hi].copy()
        sub_ll = ll[lo:hi].copy()
        sub_fl = fl[offs[lo]:offs[hi]].copy()
        shards.append((np.ascontiguousarray(f[:, lo:hi]), sub_nf, sub_fl, sub_ll))
    return (f, nf, fl, ll), shards


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_lib as oracle
    from conftest import load_kctc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    kctc = load_kctc()
    R, H, D, A, T, N = 2, 8, 6, 7, 15, 4
    _, shards = _split(kctc, T, N, D, A, 77)
    # both shards keep utterance 0's T_max so padding is identical (no masking)
    f, nf, fl, ll = shards[rank]
    grads, stats = _shard_grads(oracle, f, nf, fl, ll, R, H, D, A)
    flat = torch.from_numpy(np.concatenate([g.ravel() for g in grads]))
    dist.all_reduce(flat)           # the RCCL SUM all-reduce, here over gloo
    st = torch.from_numpy(stats)
    dist.all_reduce(st)             # sum of costs / accuracy / weight
    if rank == 0:
        q.put((flat.numpy(), st.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_sum_allreduce_equals_concatenated_minibatch(kctc, oracle):
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    flat, stats = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    R, H, D, A, T, N = 2, 8, 6, 7, 15, 4
    (f, nf, fl, ll), _ = _split(kctc, T, N, D, A, 77)
    grads, full_stats = _shard_grads(oracle, f, nf, fl, ll, R, H, D, A)
    ref = np.concatenate([g.ravel() for g in grads])
    np.testing.assert_allclose(flat, ref, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(stats, full_stats, rtol=1e-12)
