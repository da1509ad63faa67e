"""SpliceComponent with frame context (src/nnet2/nnet-component.cc:2504-2820)
and FormatNnetInput's num_splice > 1 layout (src/ctc/ctc-nnet-update.cc:351-424)
on the GPU.

With left / right context L / R the network input of a minibatch has
num_splice = 1 + L + R rows per output frame: row (t*N + n)*num_splice + s =
input frame t + s of utterance n (zero rows past its frames), and the Splice
output of frame (t, n) concatenates rows L + context[c] of that chunk.  The
oracle has no splice of its own (Splice is identity in its topology), so it
is fed the same spliced frames directly: x'[t, n] = [x_n[t + L + c] for c in
context], into a first RNN of input dim |context| * D.  Tolerance as the
other train-step tests: objective 1e-5, parameters 1e-5 relative."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _spec(oracle, R, H, Din, A, lr):
    s = oracle.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = R, 2, H, 2, 1
    s.input_dim, s.num_targets = Din, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, lr, lr
    return s


def _minibatch(rng, N, T, D, A, L, R):
    """Per-utterance input frames (T_n + L + R each), the FormatNnetInput
    layout and the oracle's pre-spliced [T, N, |ctx| D] view are built by the
    caller from these."""
    Tn = [T - int(rng.integers(0, T // 4)) if n else T for n in range(N)]
    xs = [rng.standard_normal((t + L + R, D)).astype(np.float32) for t in Tn]
    labels = []
    for t in Tn:
        lab, prev = [], -1
        for _ in range(max(1, t // 6)):
            v = int(rng.integers(1, A))
            while v == prev:
                v = int(rng.integers(1, A))
            lab.append(v)
            prev = v
        labels.append(lab)
    return Tn, xs, labels


def _format(xs, Tn, T, N, ns):
    D = xs[0].shape[1]
    out = np.zeros((T * N * ns, D), np.float32)
    for n, (x, t_n) in enumerate(zip(xs, Tn)):
        for t in range(t_n):
            for s in range(ns):
                out[(t * N + n) * ns + s] = x[t + s]
    return out


def _spliced(xs, Tn, T, N, ctx, L):
    D = xs[0].shape[1]
    out = np.zeros((T, N, len(ctx) * D), np.float64)
    for n, (x, t_n) in enumerate(zip(xs, Tn)):
        for t in range(t_n):
            out[t, n] = np.concatenate([x[t + L + c] for c in ctx])
    return out


@pytest.mark.parametrize("ctx", [(-1, 0, 1), (-2, 0, 1), (0, 2)])
def test_spliced_train_steps_match_oracle(kctc, gpu, oracle, ctx):
    import torch
    L, R = -ctx[0], ctx[-1]
    ns = 1 + L + R
    D, A, T, N, H, lr, steps, nr = 12, 11, 30, 4, 64, 0.02, 2, 2
    cfg = kctc.recipe_config(num_rnn=nr, input_dim=D, hidden=H, num_targets=A, learning_rate=lr, param_stddev=0.2,
                             splice_context=ctx)
    net = kctc.Nnet(cfg, seed=5)
    assert net.context == (L, R)
    upd = [c for c in range(net.num_components) if net.num_params(c) > 0]
    params = [net.get_params(c).astype(np.float64) for c in upd]
    spec = _spec(oracle, nr, H, len(ctx) * D, A, lr)
    rng = np.random.default_rng(sum(ctx) + 7)
    for step in range(steps):
        Tn, xs, labels = _minibatch(rng, N, T, D, A, L, R)
        nf = np.array(Tn, np.int32)
        fl = np.array([v for lab in labels for v in lab], np.int32)
        ll = np.array([len(lab) for lab in labels], np.int32)
        feats = torch.from_numpy(_format(xs, Tn, T, N, ns)).to(gpu)
        objf, acc, wt = net.train_step(feats, T, N, nf, fl, ll)
        Wa = params[-1][:-A].reshape(A, -1).copy()
        ba = params[-1][-A:].copy()
        robjf, _, rwt = oracle.train_step(spec, params[:-1], Wa, ba, _spliced(xs, Tn, T, N, ctx, L), nf, fl, ll,
                                          repair_draws=np.ones(nr, np.float32))
        params[-1] = np.concatenate([Wa.ravel(), ba])
        np.testing.assert_allclose(objf, robjf, rtol=1e-5)
        assert wt == rwt
    for c, p in zip(upd, params):
        assert rel_err(net.get_params(c).astype(np.float64), p) < 1e-5, c
    net.close()


def test_spliced_egs_format_and_train_simple(kctc, gpu, oracle, tmp_path):
    """The egs path with context: examples stored with left_context L + 1
    (one frame ignored, ignore_frames = left_context - L), the reader opened
    with the network's (L, R); the GPU FormatNnetInput equals the layout built
    from the codec restatement's decode bit for bit, num_frames are the CTC
    input lengths (NumFrames - left_context - R), and TrainNnetSimple on the
    reader equals formatting + stepping minibatch by minibatch."""
    import torch
    ctx = (-2, -1, 0, 1)
    L, R = 2, 1
    ns = 1 + L + R
    D, A, H = 16, 11, 32
    rng = np.random.default_rng(3)
    path = str(tmp_path / "ctx.ark")
    frames = []
    with kctc.EgsWriter(path) as w:
        for i in range(7):
            F = int(rng.integers(30, 60))
            x = rng.standard_normal((F, D)).astype(np.float32)
            lab = rng.integers(1, A, size=max(1, F // 8)).astype(np.int32)
            w.write(f"u{i}", x, lab, left_context=L + 1)
            frames.append(oracle.cm_decompress(oracle.cm_compress(x)))
    cfg = kctc.recipe_config(num_rnn=2, input_dim=D, hidden=H, num_targets=A, learning_rate=0.01,
                             max_seq_length=100, splice_context=ctx)
    a, b = kctc.Nnet(cfg, seed=4), kctc.Nnet(cfg, seed=4)
    assert a.context == (L, R)
    st = a.train_simple(kctc.EgsReader(path, minibatch_size=4, max_frames=1000, nnet_left_context=L,
                                       nnet_right_context=R))
    assert st["num_egs"] == 7
    seen, tot_o = 0, 0.0
    for mb in kctc.EgsReader(path, minibatch_size=4, max_frames=1000, nnet_left_context=L, nnet_right_context=R):
        assert mb.num_splice == ns
        dec = frames[seen:seen + mb.N]
        seen += mb.N
        ignore = (L + 1) - L
        tn = [x.shape[0] - ns - ignore + 1 for x in dec]
        np.testing.assert_array_equal(mb.num_frames, tn)
        assert mb.T_max == max(tn)
        feats = torch.empty((mb.T_max * mb.N * ns, mb.input_dim), dtype=torch.float32, device=gpu)
        scratch = torch.empty(mb.scratch_bytes(), dtype=torch.uint8, device=gpu)
        mb.format(feats, scratch, stream=b.stream)
        torch.cuda.synchronize()
        want = _format([x[ignore:] for x in dec], tn, mb.T_max, mb.N, ns)
        np.testing.assert_array_equal(feats.cpu().numpy(), want)
        o, _, _ = b.train_step(feats, mb.T_max, mb.N, mb.num_frames, mb.flat_labels, mb.label_lengths)
        tot_o += o
    np.testing.assert_allclose(st["tot_objf"], tot_o, rtol=1e-12)
    for c in range(a.num_components):
        if a.num_params(c):
            np.testing.assert_array_equal(a.get_params(c), b.get_params(c))
    # a reader opened with another context than the network's is refused
    with pytest.raises(kctc.KctcError):
        a.train_simple(kctc.EgsReader(path, minibatch_size=4, max_frames=1000))
    a.close()
    b.close()


@pytest.mark.parametrize("binary", [False, True])
def test_spliced_model_round_trip(kctc, gpu, tmp_path, binary):
    cfg = kctc.recipe_config(num_rnn=1, input_dim=8, hidden=32, num_targets=5, splice_context=(-3, 0, 2))
    net = kctc.Nnet(cfg, seed=2)
    p = tmp_path / "m.nnet"
    net.write(p, binary=binary)
    back = kctc.Nnet.read(p)
    assert back.context == (3, 2)
    assert back.info(0) == net.info(0) and "output-dim=24" in back.info(0)
    for c in range(net.num_components):
        if net.num_params(c):
            if binary:
                np.testing.assert_array_equal(back.get_params(c), net.get_params(c))
            else:  # Kaldi text mode writes 7 significant digits
                np.testing.assert_allclose(back.get_params(c), net.get_params(c), rtol=1e-6, atol=1e-9)
    back.close()
    net.close()
