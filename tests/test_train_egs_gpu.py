"""TrainNnetSimple over egs archives and momentum (include/kaldi_ctc_train.h:
kctc_nnet_train_simple, kctc_nnet_set_momentum) on the GPU.

* train_simple == the same minibatches formatted on the GPU and stepped one by
  one (bit-identical parameters: same kernels, same order).
* momentum vs the fp64 oracle: the oracle's step gives the SGD update
  u = lr * clip(grad) for the current parameters; the reference's delta-nnet
  recursion (src/ctc/ctc-nnet-train.cc:194-245: delta += u; W += delta;
  delta *= m) is applied on top in Python.  Self-repair is off in both (the
  model's own clip counters stay 0 under momentum, ctc-nnet-train.cc:194-202 +
  nnet-cudnn-component.cc:988-991).  Tolerance: parameter changes within 1e-4
relative norm-wise per component (north_star: grads within 1e-4).
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _write_egs(kctc, path, rng, n, D=24, A=11, T=(30, 60)):
    with kctc.EgsWriter(path) as w:
        for i in range(n):
            t = int(rng.integers(*T))
            L = int(rng.integers(1, max(2, t // 6)))
            lab = rng.integers(1, A, size=L).astype(np.int32)
            w.write(f"u{i}", rng.standard_normal((t, D)).astype(np.float32), lab)


def test_train_simple_equals_stepwise(kctc, gpu, tmp_path):
    import torch
    rng = np.random.default_rng(11)
    path = str(tmp_path / "e.ark")
    _write_egs(kctc, path, rng, 11)
    cfg = kctc.recipe_config(num_rnn=2, input_dim=24, hidden=32, num_targets=11, learning_rate=0.01,
                             max_seq_length=100)
    a = kctc.Nnet(cfg, seed=4)
    b = kctc.Nnet(cfg, seed=4)
    a.srand(5)
    b.srand(5)
    r = kctc.EgsReader(path, minibatch_size=4, max_frames=1000)
    st = a.train_simple(r)
    assert st["num_egs"] == 11
    tot_o = tot_w = 0.0
    for mb in kctc.EgsReader(path, minibatch_size=4, max_frames=1000):
        feats = torch.empty((mb.T_max * mb.N, mb.input_dim), dtype=torch.float32, device=gpu)
        scratch = torch.empty(mb.scratch_bytes(), dtype=torch.uint8, device=gpu)
        mb.format(feats, scratch, stream=b.stream)
        o, acc, w = b.train_step(feats, mb.T_max, mb.N, mb.num_frames, mb.flat_labels, mb.label_lengths)
        tot_o += o
        tot_w += w
    np.testing.assert_allclose(st["tot_objf"], tot_o, rtol=1e-12)
    assert st["tot_weight"] == tot_w
    for c in range(a.num_components):
        if a.num_params(c):
            np.testing.assert_array_equal(a.get_params(c), b.get_params(c))


@pytest.mark.parametrize("m", [0.0, 0.5, 0.9])
def test_momentum_matches_oracle(kctc, gpu, oracle, m):
    import torch
    R, D, A, T, N, lr, H = 2, 24, 11, 30, 4, 0.02, 48
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=lr,
                             param_stddev=0.2)
    net = kctc.Nnet(cfg, seed=8)
    net.set_momentum(m)
    upd = [c for c in range(net.num_components) if net.num_params(c) > 0]
    W = [net.get_params(c).astype(np.float64) for c in upd]
    W0 = [w.copy() for w in W]
    delta = [np.zeros_like(w) for w in W]
    s = oracle.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = R, 2, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, lr, lr
    for step in range(3):
        feats, nf, fl, ll = kctc.synth_minibatch(500 + step, T, N, D, A, 0.2)
        objf, _, _ = net.train_step(torch.from_numpy(feats).to(gpu), T, N, nf, fl, ll)
        # oracle: SGD update at the current parameters
        rnn_p = [w.copy() for w in W[:-1]]
        Wa = W[-1][:-A].reshape(A, -1).copy()
        ba = W[-1][-A:].copy()
        robjf, _, _ = oracle.train_step(s, rnn_p, Wa, ba, feats.reshape(T, N, D).astype(np.float64), nf, fl, ll,
                                        repair_draws=np.ones(R, np.float32))
        np.testing.assert_allclose(objf, robjf, rtol=1e-5)
        new = rnn_p + [np.concatenate([Wa.ravel(), ba])]
        for i in range(len(W)):
            delta[i] = delta[i] + (new[i] - W[i])
            W[i] = W[i] + delta[i]
            delta[i] = m * delta[i]
    for c, w, w0 in zip(upd, W, W0):
        assert rel_err(net.get_params(c).astype(np.float64) - w0, w - w0) < 1e-4, c


def test_momentum_rejects_bad_value(kctc, gpu):
    net = kctc.Nnet(kctc.recipe_config(num_rnn=1, input_dim=8, hidden=16, num_targets=5), seed=1)
    with pytest.raises(kctc.KctcError):
        net.set_momentum(1.0)
