"""SURVEY §8f row 3 on the GPU: SoftmaxComponent, the CtcDecodableAmNnet
log-likelihood matrix (src/ctc/ctc-decodable-am-nnet.cc:28-80) and the
nnet2-ctc-compute-prob loop (src/ctcbin/nnet2-ctc-compute-prob.cc:27-111),
against the oracle restatements (oracle_softmax_rows_f32,
oracle_ctc_decodable_f32, oracle_train_step at lr 0).

Tolerances: softmax 5e-6 relative (fp32 rounding of x - max, then exp); the decodable
matrix is compared on the GPU's own probabilities (same floats in), so only
logf rounding separates them: 1e-6 relative, kept rows bit-exact."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(180)]


def test_softmax_rows_matches_oracle(kctc, gpu, oracle):
    import torch
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((5000, 41)) * 8).astype(np.float32)
    x[0] = 0.0
    x[1, 5] = 80.0                      # saturated row: the others floor at 1e-20
    x[2] = -1e4
    y = kctc.softmax_rows(torch.from_numpy(x).to(gpu)).cpu().numpy()
    ref = oracle.softmax_rows(x)
    # fp32 x - max rounds by up to ulp(|x - max|) / 2 (~2e-6 at 40): exp inherits it
    np.testing.assert_allclose(y, ref, rtol=5e-6, atol=1e-26)
    assert y.min() >= 1e-20
    np.testing.assert_allclose(y.sum(1), 1.0, rtol=1e-5)


@pytest.mark.parametrize("blank_threshold", [1.0, 0.5, 0.2, 1e-9])
@pytest.mark.parametrize("floor", [1e-10, 1e-20])
def test_ctc_decodable_matches_oracle(kctc, gpu, oracle, blank_threshold, floor):
    import torch
    rng = np.random.default_rng(int(blank_threshold * 100) + 7)
    T, A = 1500, 41
    logits = rng.standard_normal((T, A)).astype(np.float32) * 3
    logits[:, 0] += 2.0  # blank-heavy frames, as a trained CTC model gives
    probs = kctc.softmax_rows(torch.from_numpy(logits).to(gpu))
    priors = (rng.random(A) + 0.01).astype(np.float32)
    priors /= priors.sum()
    for pr in (None, priors):
        out = kctc.ctc_decodable(probs, None if pr is None else torch.from_numpy(pr).to(gpu), prob_scale=0.7,
                                 blank_threshold=blank_threshold, floor=floor).cpu().numpy()
        ref = oracle.ctc_decodable(probs.cpu().numpy(), pr, 0.7, blank_threshold, floor)
        assert out.shape == ref.shape
        np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-5)
    if blank_threshold == 1e-9:  # nothing qualifies: every frame is kept (:59-61)
        assert out.shape[0] == T
    if blank_threshold == 0.5:
        assert 0 < out.shape[0] < T


def _decode_cfg(kctc, D, H, A):
    return kctc.recipe_config(num_rnn=2, input_dim=D, hidden=H, num_targets=A, param_stddev=0.1) + \
        f"SoftmaxComponent dim={A}\n"


def test_decode_model_end_to_end(kctc, gpu, oracle, tmp_path):
    """A decode model (training topology + SoftmaxComponent, as nnet-insert
    leaves it) through NnetComputation and CtcDecodableAmNnet with priors."""
    import torch
    D, H, A, T = 40, 64, 11, 300
    net = kctc.Nnet(_decode_cfg(kctc, D, H, A), seed=9)
    assert "SoftmaxComponent" in net.info(net.num_components - 1)
    rng = np.random.default_rng(5)
    priors = (rng.random(A) + 0.05).astype(np.float32)
    priors /= priors.sum()
    net.set_priors(priors)
    feats = rng.standard_normal((T, D)).astype(np.float32)
    f = torch.from_numpy(feats).to(gpu)
    probs = net.propagate(f, T, 1).cpu().numpy()
    # forward vs the fp64 oracle (RNN -> RNN -> affine -> softmax)
    x = feats.reshape(T, 1, D).astype(np.float64)
    for c in (1, 3):
        x, _ = oracle.rnn_forward(2, x, net.get_params(c).astype(np.float64), H, 1, 2)
    aff = net.get_params(5).astype(np.float64)
    logits = x.reshape(T, -1) @ aff[:-A].reshape(A, -1).T + aff[-A:]
    assert rel_err(probs, oracle.softmax_rows(logits.astype(np.float32))) < 1e-5
    out = net.decodable(f, T, prob_scale=0.9, blank_threshold=0.4)
    ref = oracle.ctc_decodable(probs, priors, 0.9, 0.4, 1e-10)
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-5)
    # model file with the SoftmaxComponent: write, read, byte-identical write-back
    p1, p2 = tmp_path / "dec.mdl", tmp_path / "dec2.mdl"
    net.write_am(p1, binary=True)
    n2 = kctc.Nnet.read_am(p1)
    n2.write_am(p2, binary=True)
    assert p1.read_bytes() == p2.read_bytes()
    np.testing.assert_array_equal(n2.decodable(f, T, 0.9, 0.4), out)
    n2.close()
    net.close()


def test_compute_prob_matches_batches_and_oracle(kctc, gpu, oracle, tmp_path):
    """nnet2-ctc-compute-prob: batches of 10 examples in archive order, no
    training skip rules (one example is longer than max_allow_frames)."""
    import torch
    D, H, A, R = 40, 64, 11, 2
    rng = np.random.default_rng(11)
    path = str(tmp_path / "valid.egs")
    egs = []
    with kctc.EgsWriter("ark:" + path) as w:
        for i in range(23):
            T = 2100 if i == 13 else int(rng.integers(20, 90))
            L = int(rng.integers(1, max(2, T // 6)))
            lab = rng.integers(1, A, L).astype(np.int32)
            feats = rng.standard_normal((T, D)).astype(np.float32)
            w.write(f"utt{i:03d}", feats, lab)
            egs.append((oracle.cm_decompress(oracle.cm_compress(feats)), lab))
    net = kctc.Nnet(kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, param_stddev=0.1), seed=2)
    res = net.compute_prob("ark:" + path)
    assert res["num_examples"] == 23
    tot = np.zeros(3)
    rtot = np.zeros(2)
    s = oracle.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = R, 2, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, 0.0, 0.0
    params = [net.get_params(c).astype(np.float64) for c in (1, 3, 5)]
    for b0 in range(0, 23, 10):
        batch = egs[b0:b0 + 10]
        feats = kctc.format_input([e[0] for e in batch])
        T = feats.shape[0] // len(batch)
        nf = np.array([e[0].shape[0] for e in batch], np.int32)
        fl = np.concatenate([e[1] for e in batch])
        ll = np.array([len(e[1]) for e in batch], np.int32)
        o, a, wt = net.compute_objf(torch.from_numpy(feats).to(gpu), T, len(batch), nf, fl, ll)
        tot += (o, a, wt)
        Wa, ba = params[2][:-A].reshape(A, -1).copy(), params[2][-A:].copy()
        ro, _, _ = oracle.train_step(s, [p.copy() for p in params[:2]], Wa, ba,
                                     feats.reshape(T, len(batch), D).astype(np.float64), nf, fl, ll)
        rtot[0] += ro
        rtot[1] += wt
    # the same per-batch ComputeNnetObjf sums (host-formatted vs GPU-formatted input)
    np.testing.assert_allclose([res["tot_like"], res["tot_accuracy"], res["tot_weight"]], tot, rtol=1e-6)
    np.testing.assert_allclose(res["tot_like"], rtot[0], rtol=1e-5)
    assert res["tot_weight"] == rtot[1]
    net.close()


@pytest.mark.parametrize("ctx", [(-2, 0, 1), (0, 3)])
def test_decode_spliced_model_pads_input(kctc, gpu, oracle, ctx):
    """CtcDecodableAmNnet(pad_input = true) of a model with frame context: the
    utterance's first / last frame repeated LeftContext / RightContext times
    (NnetComputer, src/nnet2/nnet-compute.cc:64-90) -- T frames in, T rows
    out -- vs the oracle on the same padded, spliced frames."""
    import torch
    D, H, A, T = 12, 64, 11, 150
    L, R = -ctx[0], ctx[-1]
    net = kctc.Nnet(kctc.recipe_config(num_rnn=2, input_dim=D, hidden=H, num_targets=A, param_stddev=0.1,
                                       splice_context=ctx) + f"SoftmaxComponent dim={A}\n", seed=4)
    assert net.context == (L, R)
    rng = np.random.default_rng(8)
    feats = rng.standard_normal((T, D)).astype(np.float32)
    f = torch.from_numpy(feats).to(gpu)
    out = net.decodable(f, T, prob_scale=1.0, blank_threshold=1.0)
    assert out.shape == (T, A)
    padded = np.concatenate([np.repeat(feats[:1], L, 0), feats, np.repeat(feats[-1:], R, 0)])
    x = np.stack([np.concatenate([padded[t + L + c] for c in ctx]) for t in range(T)])
    x = x.reshape(T, 1, -1).astype(np.float64)
    for c in (1, 3):
        x, _ = oracle.rnn_forward(2, x, net.get_params(c).astype(np.float64), H, 1, 2)
    aff = net.get_params(5).astype(np.float64)
    logits = x.reshape(T, -1) @ aff[:-A].reshape(A, -1).T + aff[-A:]
    ref = oracle.ctc_decodable(oracle.softmax_rows(logits.astype(np.float32)), None, 1.0, 1.0, 1e-10)
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=2e-5)
    # the trainer's own input check: a [T, D] buffer is not a spliced network's layout
    with pytest.raises(kctc.KctcError):
        net.propagate(f, T, 1)
    net.close()
