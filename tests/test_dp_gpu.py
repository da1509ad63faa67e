"""Data parallelism through the product trainer: two ranks, each a
process with its own nnet2 trainer on the one GPU of the box, exchange their
gradient buckets through kctc_nnet_enable_dp_host (gloo all-reduce on the
host; the same GradExchange hook, bucket order and sum -> +-5 clip -> SGD
path as the RCCL exchange).  Semantics under test: the summed gradient of the
two per-rank minibatches is the gradient of their concatenation, so both
replicas end bit-identical to each other and equal (to fp32 summation order)
to ONE trainer stepping on the concatenated minibatch; the rand() stream of
self-repair is drawn identically on every rank (one RandUniform() per
ClipGradient Backprop), while the clip counters stay per rank."""
import os
import sys

import numpy as np
import pytest

from conftest import rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D, A, T, N, H, R, STEPS = 40, 41, 48, 4, 256, 2, 2


def _cfg(kctc):
    return kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=1e-3,
                              param_stddev=0.05)


def _batch(kctc, rank, step):
    return kctc.synth_minibatch(500 + 10 * step + rank, T, N, D, A, 0.125)


def _rank_main(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        kctc = ge.load_package()
        net = kctc.Nnet(_cfg(kctc), seed=21)

        def allreduce(buf):
            t = torch.from_numpy(buf)  # shares the pinned buffer
            dist.all_reduce(t)

        net.enable_dp_host(allreduce, world)
        stats = []
        for step in range(STEPS):
            feats, nf, fl, ll = _batch(kctc, rank, step)
            stats.append(net.train_step(torch.from_numpy(feats).to("cuda:0"), T, N, nf, fl, ll))
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        clip = [net.clip_stats(c) for c in range(net.num_components) if "ClipGradient" in net.info(c)]
        q.put((rank, stats, params, clip, net.rand_calls))
        net.close()
        dist.destroy_process_group()
    except BaseException as e:  # report, never hang the parent
        q.put((rank, repr(e), None, None, None))


def test_two_rank_dp_equals_concatenated_minibatch(kctc, gpu):
    import torch
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 2000
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=200)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r][2] is not None, res[r][1]
    # replicas identical after every update
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)
    # same draws on every rank, counters per rank
    assert res[0][4] == res[1][4] == STEPS * R
    for (c0, n0), (c1, n1) in zip(res[0][3], res[1][3]):
        assert n0 == n1 == STEPS * T * N
    # one trainer on the concatenation of the two ranks' minibatches
    net = kctc.Nnet(_cfg(kctc), seed=21)
    for step in range(STEPS):
        b = [_batch(kctc, r, step) for r in (0, 1)]
        feats = np.concatenate([x[0].reshape(T, N, D) for x in b], axis=1).reshape(T * 2 * N, D)
        nf = np.concatenate([x[1] for x in b])
        fl = np.concatenate([x[2] for x in b])
        ll = np.concatenate([x[3] for x in b])
        o, acc, w = net.train_step(torch.from_numpy(np.ascontiguousarray(feats)).to(gpu), T, 2 * N, nf, fl, ll)
        o0, a0, w0 = res[0][1][step]
        o1, a1, w1 = res[1][1][step]
        np.testing.assert_allclose(o, o0 + o1, rtol=1e-5)  # objective of the concatenation
        assert w == w0 + w1
    ref = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
    for a, b in zip(res[0][2], ref):
        assert rel_err(a.astype(np.float64), b.astype(np.float64)) < 1e-6
    net.close()


def _avg_rank_main(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        kctc = ge.load_package()
        net = kctc.Nnet(_cfg(kctc), seed=21)

        def allreduce(buf):
            dist.all_reduce(torch.from_numpy(buf))

        net.set_dp_mode("average")
        net.enable_dp_host(allreduce, world)
        for step in range(STEPS):
            feats, nf, fl, ll = _batch(kctc, rank, step)
            net.train_step(torch.from_numpy(feats).to("cuda:0"), T, N, nf, fl, ll)
        before = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.average_params()
        after = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        q.put((rank, before, after))
        net.close()
        dist.destroy_process_group()
    except BaseException as e:  # report, never hang the parent
        q.put((rank, repr(e), None))


def test_two_rank_model_averaging(kctc, gpu):
    """kctc_nnet_set_dp_mode(1): the ranks step independently (no gradient
    exchange), then kctc_nnet_average_params makes every updatable
    component the mean of the ranks' copies -- the recipe's nnet-am-average
    (nnet-am-average.cc:185-241, weights 1/2).  Each rank's pre-average
    parameters equal a lone trainer on that rank's minibatches; afterwards
    both ranks hold (p0 + p1) / 2 bit for bit."""
    import torch
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 2000
    procs = [ctx.Process(target=_avg_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=200)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r][2] is not None, res[r][1]
    for r in (0, 1):  # independent steps: a lone trainer on rank r's data
        net = kctc.Nnet(_cfg(kctc), seed=21)
        for step in range(STEPS):
            feats, nf, fl, ll = _batch(kctc, r, step)
            net.train_step(torch.from_numpy(feats).to(gpu), T, N, nf, fl, ll)
        alone = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.close()
        for a, b in zip(res[r][1], alone):
            np.testing.assert_array_equal(a, b)
    for p0, p1, a0, a1 in zip(res[0][1], res[1][1], res[0][2], res[1][2]):
        np.testing.assert_array_equal(a0, a1)
        np.testing.assert_array_equal(a0, (p0 + p1) * np.float32(0.5))


def _fail_rank_main(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        kctc = ge.load_package()
        net = kctc.Nnet(_cfg(kctc), seed=21)

        def allreduce(buf):
            dist.all_reduce(torch.from_numpy(buf))

        net.enable_dp_host(allreduce, world)
        params, errors = [], []
        for step in range(3):
            feats, nf, fl, ll = _batch(kctc, rank, step)
            if step == 1 and rank == 1:
                net.inject_step_error(1)  # as if rank 1's recurrence had timed out
            try:
                net.train_step(torch.from_numpy(feats).to("cuda:0"), T, N, nf, fl, ll)
                errors.append(None)
            except Exception as e:  # noqa: BLE001 -- the failed step raises on every rank
                errors.append(str(e))
            params.append([net.get_params(c) for c in range(net.num_components) if net.num_params(c)])
        q.put((rank, errors, params))
        net.close()
        dist.destroy_process_group()
    except BaseException as e:  # report, never hang the parent
        q.put((rank, repr(e), None))


def test_failed_step_on_one_rank_is_skipped_on_all(kctc, gpu):
    """a step whose device error word is set on ONE rank
    must not be applied anywhere -- the gradients were already summed into
    every rank's buffers.  The word is summed over the ranks before the
    updates: both ranks skip step 1 (parameters equal to after step 0), both
    raise, the local rank with the timeout message and the other with the
    peer message, and the replicas stay bit-identical through step 2."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + os.getpid() % 2000
    procs = [ctx.Process(target=_fail_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=200)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r][2] is not None, res[r][1]
    e0, e1 = res[0][1], res[1][1]
    assert e0[0] is None and e1[0] is None and e0[2] is None and e1[2] is None
    assert e1[1] is not None and "timed out" in e1[1]
    assert e0[1] is not None and "another data-parallel rank" in e0[1]
    for r in (0, 1):
        for a, b in zip(res[r][2][0], res[r][2][1]):
            np.testing.assert_array_equal(a, b)  # step 1 skipped
    for step in range(3):
        for a, b in zip(res[0][2][step], res[1][2][step]):
            np.testing.assert_array_equal(a, b)  # replicas identical
    assert any(np.any(a != b) for a, b in zip(res[0][2][1], res[0][2][2]))  # step 2 applied
