"""The reference's generic component gradient check, run on the HIP components.

UnitTestGenericComponentInternal (src/nnet2/nnet-component-test.cc:28-208)
restated step for step through the Component C ABI
(include/kaldi_nnet2_component.h):

  * random input, a random objective vector `objf_vec`; objf = sum over output
    rows of output . objf_vec (a linear function of the output);
  * Write the component (text or binary at random) and ReadNew a copy;
  * input derivative: the copy's Backprop with out_deriv = objf_vec in every
    row; ten times perturb the input by 1e-4 * N(0,1) and compare the
    predicted change TraceMatMat(delta, in_deriv) with the observed change of
    objf -- bad when they differ by more than 15 % of their mean and 1e-6;
  * parameter derivative (UpdatableComponents): ten times copy the component
    twice, SetZero(true) one copy (the gradient holder: learning rate 1),
    PerturbParams(5e-4) the other, Backprop with the gradient holder as
    to_update, and compare perturbed.DotProduct(grad) - orig.DotProduct(grad)
    with the observed change of objf -- 5 % and 1e-6.

The reference's check passes with its own rule (the input check fails when
the bad tries are at least half, the model check when they are a majority).
At recipe width its one-sided differences carry two errors that have nothing
to do with the derivative: the curvature term (a 5e-4 perturbation of all
2.3 M parameters of a BLSTM-512 moves the objective by up to 5 % of the
first-order term in fp64, measured with torch on the CPU) and fp32-class
rounding of the ~50 k output values at a 1e-4 input step (a few %).  So every
derivative is also checked by central differences -- input step 1e-2, model
step 5e-4, the curvature term cancelling -- and there all ten tries must be
within 1 % of the larger of |predicted| and its rms over random directions
(step * |derivative|: a direction nearly orthogonal to the derivative makes
the predicted change arbitrarily small, and any relative error with it).  The worst errors go to gpurun_out/component_gradcheck.txt (and
stdout under -s).  The objective sums run in fp64 on the device (the
reference: fp32 AddMatVec + Sum); the components compute exactly as in
training.

Differences from the reference's driver, all on the test side:
  * CuDNNRecurrentComponent Backprop needs the reserve space of a Propagate of
    the same component on the same input (cuDNN's contract,
    nnet-cudnn-component.cc:558-599), so the read-back copy is propagated once
    before its Backprop (the reference's CPU-only test never runs this
    component);
  * the recurrent components use clip-gradient=1e30 in the parameter check:
    the reference clips dW to +-5 before the update (:602-603), which the
    gradient holder would otherwise receive clipped (the objective here is a
    sum over every frame, so dW entries exceed 5);
  * the recurrences run in their fp32-class arithmetic; the bf16 path
    (configs[4]) rounds operands to 8 bits, far coarser than a 1e-4 input
    perturbation, and is covered by the oracle tests instead;
  * SpliceComponent's input is this path's FormatNnetInput layout
    (num_splice rows per output frame), N chunks of T frames.
"""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

INPUT_TOL, PARAM_TOL = 0.15, 0.05      # nnet-component-test.cc:118-120, 186-188
CENTRAL_TOL = 0.01
LOG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out", "component_gradcheck.txt")


def _objf(out, v):
    return float((out.double() @ v.double()).sum())


def _log(line):
    print(line)
    try:
        os.makedirs(os.path.dirname(LOG), exist_ok=True)
        with open(LOG, "a") as f:
            f.write(line + "\n")
    except OSError:
        pass


def _bad(pred, obs, tol):
    return abs(pred - obs) > tol * abs((pred + obs) / 2) and abs(pred - obs) > 1e-6


def _rel(pred, obs):
    return abs(pred - obs) / max(abs((pred + obs) / 2), 1e-30)


def generic_component_check(kctc, gpu, comp, T, N, tmp_path, seed, input_scale=1.0, name="", step=1.0e-2,
                            central_tol=CENTRAL_TOL):
    """UnitTestGenericComponentInternal(component, in_info, out_info), then the
    same derivatives by central differences; returns the worst relative
    errors (reference input check, reference model check, central input,
    central model)."""
    import torch
    g = torch.Generator(device=gpu)
    g.manual_seed(seed)
    rng = np.random.default_rng(seed)
    ns = comp.NumSplice()
    rows_in, rows = T * N * ns, T * N
    inp = torch.randn((rows_in, comp.InputDim()), generator=g, device=gpu) * input_scale
    v = torch.randn((comp.OutputDim(),), generator=g, device=gpu)
    output = comp.Propagate(T, N, inp)
    binary = bool(rng.integers(2))
    path = tmp_path / f"tmpf_{seed}"
    comp.Write(path, binary=binary)
    copy = kctc.Component.ReadNew(path)
    assert copy.Type() == comp.Type() and copy.InputDim() == comp.InputDim()
    rec = copy.Type() == "CuDNNRecurrentComponent"

    # ---- input derivative ----
    objf = _objf(output, v)
    out_deriv = v.expand(rows, -1).contiguous()
    in_deriv = torch.empty_like(inp)
    needs_in, needs_out = copy.BackpropNeedsInput(), copy.BackpropNeedsOutput()
    if rec:
        copy.Propagate(T, N, inp)  # the reserve space its Backprop reads
    copy.Backprop(T, N, inp if needs_in else None, output if needs_out else None, out_deriv, None, in_deriv)
    worst_in = worst_inc = 0.0
    bad = bad_c = 0
    # rms of the predicted change over random directions: delta . in_deriv with
    # delta ~ N(0, I) has standard deviation |in_deriv|
    rms_in = float(in_deriv.double().norm())
    for _ in range(10):
        delta = torch.randn(inp.shape, generator=g, device=gpu)
        predicted = float((delta.double() * in_deriv.double()).sum())
        obs = _objf(comp.Propagate(T, N, (delta * 1.0e-4 + inp).contiguous()), v) - objf
        worst_in = max(worst_in, _rel(predicted * 1.0e-4, obs))
        bad += _bad(predicted * 1.0e-4, obs, INPUT_TOL)
        # central difference at `step` (1e-2): the curvature term cancels, fp32
        # noise is 100x smaller
        obs_c = (_objf(comp.Propagate(T, N, (delta * step + inp).contiguous()), v) -
                 _objf(comp.Propagate(T, N, (inp - delta * step).contiguous()), v)) / 2
        err_c = abs(predicted * step - obs_c) / max(abs(predicted * step), step * rms_in)
        worst_inc = max(worst_inc, err_c)
        bad_c += err_c > central_tol
    _log(f"{name}: input gradients  reference check worst rel err {worst_in:.3e} ({10 - bad}/10 within "
         f"{INPUT_TOL}); central worst {worst_inc:.3e}")
    assert bad < 5, f"{name}: feature-derivative check failed ({bad}/10 bad, worst {worst_in:.3g})"
    assert bad_c == 0, f"{name}: central input derivative off by {worst_inc:.3g}"

    worst_p = worst_pc = None
    if copy.IsUpdatable():
        worst_p = worst_pc = 0.0
        bad = bad_c = 0
        for _ in range(10):
            perturbed, grad = copy.Copy(), copy.Copy()
            grad.SetZero(True)
            assert grad.IsGradient() and grad.LearningRate() == 1.0
            perturbed.PerturbParams(5.0e-4)
            if rec:
                copy.Propagate(T, N, inp)
            copy.Backprop(T, N, inp, output, out_deriv, grad, torch.empty_like(inp))
            f_plus = _objf(perturbed.Propagate(T, N, inp), v)
            observed = f_plus - objf
            predicted = perturbed.DotProduct(grad) - copy.DotProduct(grad)
            worst_p = max(worst_p, _rel(predicted, observed))
            bad += _bad(predicted, observed, PARAM_TOL)
            # central: theta - delta = 2 theta - (theta + delta)
            minus = copy.Copy()
            minus.Scale(2.0)
            minus.Add(-1.0, perturbed)
            obs_c = (f_plus - _objf(minus.Propagate(T, N, inp), v)) / 2
            # normalised like the input check: the rms of delta . grad over
            # directions is 5e-4 |grad|
            err_c = abs(predicted - obs_c) / max(abs(predicted), 5.0e-4 * np.sqrt(grad.DotProduct(grad)))
            worst_pc = max(worst_pc, err_c)
            bad_c += err_c > central_tol
            for x in (perturbed, grad, minus):
                x.close()
        _log(f"{name}: model gradients reference check worst rel err {worst_p:.3e} ({10 - bad}/10 within "
             f"{PARAM_TOL}); central worst {worst_pc:.3e}")
        assert bad <= 5, f"{name}: model-derivative check failed ({bad}/10 bad, worst {worst_p:.3g})"
        assert bad_c == 0, f"{name}: central model derivative off by {worst_pc:.3g}"
    copy.close()
    return worst_in, worst_p, worst_inc, worst_pc


RNN_CASES = [
    # (name, config line, T, N)
    ("BLSTM-512 layer 1 (configs[1])",
     "CuDNNRecurrentComponent input-dim=40 output-dim=512 bidirectional=true max-seq-length=2000 "
     "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30", 12, 4),
    ("BLSTM-512 layers 2-5 (configs[1])",
     "CuDNNRecurrentComponent input-dim=1024 output-dim=512 bidirectional=true max-seq-length=2000 "
     "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30", 12, 4),
    ("BLSTM-512 N=16 row groups",
     "CuDNNRecurrentComponent input-dim=1024 output-dim=512 bidirectional=true max-seq-length=2000 "
     "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30", 6, 16),
    ("BGRU-1024 (configs[4], fp32-class)",
     "CuDNNRecurrentComponent input-dim=2048 output-dim=1024 bidirectional=true max-seq-length=2000 "
     "learning-rate=0.0005 rnn-mode=3 num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30", 8, 4),
    ("uni-LSTM-256 (configs[0])",
     "CuDNNRecurrentComponent input-dim=40 output-dim=256 bidirectional=false max-seq-length=200 "
     "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30", 10, 2),
    ("BLSTM-64 x2 layers",
     "CuDNNRecurrentComponent input-dim=24 output-dim=64 bidirectional=true max-seq-length=100 "
     "learning-rate=0.001 rnn-mode=2 num-layers=2 param-stddev=0.1 bias-stddev=0.2 clip-gradient=1e30", 9, 3),
    ("BiRNN-TANH-48",
     "CuDNNRecurrentComponent input-dim=20 output-dim=48 bidirectional=true max-seq-length=100 "
     "learning-rate=0.001 rnn-mode=1 num-layers=1 param-stddev=0.1 bias-stddev=0.2 clip-gradient=1e30", 9, 3),
    # RELU: a 1e-2 input step crosses the kinks of max(0, .); 1e-3 crosses 10x
    # fewer, and the 5e-4 parameter step still crosses some (measured 0.6 % /
    # 1.4 %): central bar 5 %
    ("BiRNN-RELU-48",
     "CuDNNRecurrentComponent input-dim=20 output-dim=48 bidirectional=true max-seq-length=100 "
     "learning-rate=0.001 rnn-mode=0 num-layers=1 param-stddev=0.1 bias-stddev=0.2 clip-gradient=1e30", 9, 3, 1e-3,
     0.05),
]


@pytest.mark.parametrize("case", RNN_CASES, ids=[c[0] for c in RNN_CASES])
def test_recurrent_component_gradients(kctc, gpu, tmp_path, case):
    name, line, T, N = case[:4]
    step = case[4] if len(case) > 4 else 1.0e-2
    central_tol = case[5] if len(case) > 5 else CENTRAL_TOL
    kctc.set_perturb_seed(101)
    comp = kctc.Component(line, seed=7)
    generic_component_check(kctc, gpu, comp, T, N, tmp_path, seed=11, name=name, step=step, central_tol=central_tol)


def test_affine_component_gradients(kctc, gpu, tmp_path):
    # UnitTestAffineComponent's InitFromString case (nnet-component-test.cc:357-361) and the
    # recipe's output layer (BLSTM-512 -> 41 targets)
    for name, line, T, N in [("Affine 10->15", "AffineComponent learning-rate=0.01 input-dim=10 output-dim=15 "
                              "param-stddev=0.1", 13, 1),
                             ("Affine 1024->41", "AffineComponent input-dim=1024 output-dim=41", 50, 16)]:
        comp = kctc.Component(line, seed=3)
        wi, wp, wic, wpc = generic_component_check(kctc, gpu, comp, T, N, tmp_path, seed=5, name=name)
        assert max(wic, wpc) < 1e-3, (name, wic, wpc)  # linear: exact up to fp32 rounding


@pytest.mark.parametrize("ctx,const_dim,feat_dim,chunks", [
    ((-2, -1, 0, 1, 2), 0, 13, 7),      # contiguous (UnitTestSpliceComponent, nnet-component-test.cc:747-809)
    ((-3, 0, 2), 4, 9, 11),             # non-contiguous with a constant part
    ((0,), 0, 40, 5),                   # the recipe's Splice (identity)
])
def test_splice_component_gradients(kctc, gpu, tmp_path, ctx, const_dim, feat_dim, chunks):
    line = (f"SpliceComponent input-dim={feat_dim + const_dim} context={':'.join(map(str, ctx))} "
            f"const-component-dim={const_dim}")
    comp = kctc.Component(line)
    assert comp.OutputDim() == feat_dim * len(ctx) + const_dim
    generic_component_check(kctc, gpu, comp, 6, chunks, tmp_path, seed=17, name=f"Splice {ctx}")


def test_softmax_component_gradients(kctc, gpu, tmp_path):
    # UnitTestGenericComponent<SoftmaxComponent> (dim=15) and the decoding output layer (dim 41)
    for dim in (15, 41):
        comp = kctc.Component(f"SoftmaxComponent dim={dim}")
        generic_component_check(kctc, gpu, comp, 12, 3, tmp_path, seed=dim, name=f"Softmax {dim}")


def test_clip_gradient_component(kctc, gpu, tmp_path):
    """Below the threshold ClipGradient is the identity both ways and passes the
    generic check; above it the backprop is the clipped derivative by design
    (nnet-cudnn-component.cc:921-970), so the predicted change is the observed
    one times min(1, threshold / |objf_vec|) exactly."""
    import torch
    comp = kctc.Component("ClipGradientComponent dim=100 clipping-threshold=30 norm-based-clipping=true")
    generic_component_check(kctc, gpu, comp, 10, 4, tmp_path, seed=23, name="ClipGradient 100 (unclipped)")
    # the recipe's line at width 1024: |objf_vec| ~ 32 > 30, every row clipped
    comp = kctc.Component("ClipGradientComponent dim=1024 clipping-threshold=30 norm-based-clipping=true")
    g = torch.Generator(device=gpu)
    g.manual_seed(29)
    T, N = 8, 4
    inp = torch.randn((T * N, 1024), generator=g, device=gpu)
    v = torch.randn((1024,), generator=g, device=gpu) * 2
    out = comp.Propagate(T, N, inp)
    assert torch.equal(out, inp)
    dy = v.expand(T * N, -1).contiguous()
    dx = torch.empty_like(inp)
    comp.Backprop(T, N, inp, None, dy, comp, dx)  # to_update = itself: the counters move
    scale = min(1.0, 30.0 / float(v.double().norm()))
    torch.testing.assert_close(dx, dy * scale, rtol=2e-6, atol=0)


def test_updatable_component_arithmetic(kctc, gpu):
    """SetZero / DotProduct / PerturbParams / Scale / Add against numpy on the
    Vectorize()d parameters (nnet-component.h:295-318)."""
    for line in ["AffineComponent input-dim=1024 output-dim=41",
                 "CuDNNRecurrentComponent input-dim=40 output-dim=512 bidirectional=true max-seq-length=2000 "
                 "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2"]:
        a, b = kctc.Component(line, seed=1), kctc.Component(line, seed=2)
        pa, pb = a.Vectorize().astype(np.float64), b.Vectorize().astype(np.float64)
        assert abs(a.DotProduct(b) - pa @ pb) <= 1e-9 * np.abs(pa * pb).sum()
        a.Scale(0.5)
        np.testing.assert_array_equal(a.Vectorize(), (pa * 0.5).astype(np.float32))
        a.Add(-2.0, b)
        np.testing.assert_allclose(a.Vectorize(), pa * 0.5 - 2.0 * pb, rtol=1e-6, atol=1e-7)
        c = b.Copy()
        np.testing.assert_array_equal(c.Vectorize(), pb.astype(np.float32))
        kctc.set_perturb_seed(9)
        c.PerturbParams(0.01)
        d = c.Vectorize().astype(np.float64) - pb
        assert abs(d.mean()) < 5 * 0.01 / np.sqrt(d.size) and abs(d.std() / 0.01 - 1) < 0.05
        c2 = b.Copy()
        kctc.set_perturb_seed(9)
        c2.PerturbParams(0.01)
        np.testing.assert_array_equal(c2.Vectorize(), c.Vectorize())   # seeded stream
        c2.PerturbParams(0.01)
        assert not np.array_equal(c2.Vectorize(), c.Vectorize())       # fresh noise per call
        lr = c.LearningRate()
        c.SetZero(False)
        assert not c.Vectorize().any() and c.LearningRate() == lr and not c.IsGradient()
        c.SetZero(True)
        assert c.LearningRate() == 1.0 and c.IsGradient()
        for x in (a, b, c, c2):
            x.close()


def test_component_text_binary_round_trip(kctc, gpu, tmp_path):
    """Component::Write / ReadNew in both modes give the same Info and the same
    parameters (bit for bit in binary mode, to the 7 digits of text mode)."""
    for line in ["AffineComponent input-dim=64 output-dim=41 learning-rate=0.001",
                 "CuDNNRecurrentComponent input-dim=40 output-dim=64 bidirectional=true max-seq-length=100 "
                 "learning-rate=0.0005 rnn-mode=3 num-layers=1 param-stddev=0.02 bias-stddev=0.2",
                 "ClipGradientComponent dim=128 clipping-threshold=30 norm-based-clipping=true",
                 "SpliceComponent input-dim=40 context=-1:0:1", "SoftmaxComponent dim=41"]:
        c = kctc.Component(line, seed=4)
        for binary in (False, True):
            p = tmp_path / f"c_{binary}"
            c.Write(p, binary=binary)
            r = kctc.Component.ReadNew(p)
            assert r.Info() == c.Info()
            if c.IsUpdatable():
                if binary:
                    np.testing.assert_array_equal(r.Vectorize(), c.Vectorize())
                else:  # Kaldi text mode writes 7 significant digits (InitKaldiOutputStream)
                    np.testing.assert_allclose(r.Vectorize(), c.Vectorize(), rtol=1e-6, atol=0)
            r.close()


def test_nnet_component_get_set_and_average(kctc, gpu):
    """Nnet::GetComponent().Copy() / SetComponent, and nnet-am-average through
    Scale / Add (nnet-am-average.cc:185-241) against numpy."""
    cfg = kctc.recipe_config(num_rnn=2, input_dim=16, hidden=32, num_targets=9)
    nets = [kctc.Nnet(cfg, seed=s) for s in (1, 2, 3)]
    upd = [c for c in range(nets[0].num_components) if nets[0].num_params(c) > 0]
    params = [[n.get_params(c).astype(np.float64) for c in upd] for n in nets]
    w = np.array([0.5, 0.3, 0.2], np.float32)
    kctc.average_models(nets, w)
    for k, c in enumerate(upd):
        ref = sum(float(w[i]) * params[i][k] for i in range(3))
        np.testing.assert_allclose(nets[0].get_params(c), ref, rtol=1e-5, atol=1e-7)
    # skip_last_layer leaves the last updatable (the affine output) alone
    a, b = kctc.Nnet(cfg, seed=1), kctc.Nnet(cfg, seed=2)
    kctc.average_models([a, b], skip_last_layer=True)
    np.testing.assert_array_equal(a.get_params(upd[-1]), params[0][-1].astype(np.float32))
    np.testing.assert_allclose(a.get_params(upd[0]), 0.5 * params[0][0] + 0.5 * params[1][0], rtol=1e-5, atol=1e-7)
    # component copies in and out of a network
    comp = b.get_component(upd[0])
    np.testing.assert_array_equal(comp.Vectorize(), b.get_params(upd[0]))
    comp.Scale(2.0)
    a.set_component(upd[0], comp)
    np.testing.assert_array_equal(a.get_params(upd[0]), comp.Vectorize())
    with pytest.raises(kctc.KctcError):
        a.set_component(upd[-1], comp)   # dimensions do not chain
    for n in nets + [a, b]:
        n.close()
    comp.close()


def test_average_models_normalises_weights(kctc, gpu):
    """GetWeights (nnet-am-average.cc:45-53) divides the weights by their sum:
    2:1 averages as 2/3 : 1/3; a weight list of the wrong length is refused."""
    cfg = kctc.recipe_config(num_rnn=1, input_dim=16, hidden=32, num_targets=9)
    nets = [kctc.Nnet(cfg, seed=s) for s in (4, 5)]
    upd = [c for c in range(nets[0].num_components) if nets[0].num_params(c) > 0]
    params = [[n.get_params(c).astype(np.float64) for c in upd] for n in nets]
    kctc.average_models(nets, [2.0, 1.0])
    for k, c in enumerate(upd):
        ref = 2.0 / 3.0 * params[0][k] + 1.0 / 3.0 * params[1][k]
        np.testing.assert_allclose(nets[0].get_params(c), ref, rtol=1e-5, atol=1e-7)
    with pytest.raises(ValueError):
        kctc.average_models(nets, [1.0])
    with pytest.raises(kctc.KctcError):
        kctc.average_models(nets, [1.0, -1.0])
    for n in nets:
        n.close()


def test_gradient_outlives_backprop_handle(kctc, gpu):
    """Kaldi's gradient-check order: Backprop into a SetZero(true) copy, destroy
    the component that ran Backprop, then DotProduct / Add on the gradient --
    the gradient must not wait on the destroyed handle's stream."""
    import torch
    line = ("CuDNNRecurrentComponent input-dim=24 output-dim=32 bidirectional=true max-seq-length=50 "
            "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2")
    comp = kctc.Component(line, seed=3)
    T, N = 10, 3
    g = torch.Generator(device=gpu)
    g.manual_seed(9)
    inp = torch.randn((T * N, 24), generator=g, device=gpu)
    out = comp.Propagate(T, N, inp)
    dy = torch.randn(out.shape, generator=g, device=gpu)
    grad = comp.Copy()
    grad.SetZero(True)
    comp.Backprop(T, N, inp, out, dy, grad, None)
    ref = comp.Copy()
    comp.close()  # its stream is gone
    d1 = grad.DotProduct(grad)
    assert np.isfinite(d1) and d1 > 0
    ref.Add(1.0, grad)
    assert np.isfinite(ref.DotProduct(grad))
    grad.close()
    ref.close()


@pytest.mark.parametrize("case", ["params_written", "other_buffers"])
def test_forward_prepacks_not_reused_when_stale(kctc, gpu, case):
    """The forward packs W^T (for the streamed dx) and x^T / y^T (for the
    weight GEMMs) beside its recurrence; Backprop reuses them only while the
    parameters are the ones packed (a parameter-version counter) and the
    in / out buffers are the ones propagated (nnet.cpp wgrad_prepack).
    params_written: Propagate, then UnVectorize new parameters, then Backprop
    -- dx and the gradient must be those of the new parameters (a reused W^T
    would give the old ones'); other_buffers: Backprop given copies of the
    propagated in / out tensors.  Reference: the same calls on a component
    without side streams (no prepack, dx after the recurrence)."""
    import torch
    T, N, D, H = 48, 16, 1024, 512
    line = (f"CuDNNRecurrentComponent input-dim={D} output-dim={H} bidirectional=true max-seq-length=200 "
            "learning-rate=0.0005 rnn-mode=2 num-layers=1 param-stddev=0.02 bias-stddev=0.2")
    g = torch.Generator().manual_seed(5)
    x = torch.tanh(torch.randn(T * N, D, generator=g)).to(gpu)
    dy = (torch.randn(T * N, 2 * H, generator=g) * 1e-2).to(gpu)

    def run(side):
        c = kctc.Component(line, seed=11)
        p1 = c.Vectorize()
        if side:
            assert kctc.lib().kctc_test_component_side_streams(c.h, 1) == 0
        y = c.Propagate(T, N, x)
        if case == "params_written":
            c.UnVectorize((p1 * 1.5).astype(np.float32))
            xin, yout = x, y
        else:
            xin, yout = x.clone(), y.clone()
        grad = c.Copy()
        grad.SetZero(True)
        dx = torch.empty_like(x)
        c.Backprop(T, N, xin, yout, dy, to_update=grad, in_deriv=dx)
        torch.cuda.synchronize()
        out = (dx.cpu().numpy().astype(np.float64), grad.Vectorize().astype(np.float64))
        grad.close()
        c.close()
        return out

    dx_s, g_s = run(True)
    dx_r, g_r = run(False)
    rel = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
    assert rel(dx_s, dx_r) < 1e-6, rel(dx_s, dx_r)
    assert rel(g_s, g_r) < 1e-6, rel(g_s, g_r)
    if case == "params_written":  # the check can tell: dx at 1.5 x W is far from dx at W
        c = kctc.Component(line, seed=11)
        y = c.Propagate(T, N, x)
        dx0 = torch.empty_like(x)
        c.Backprop(T, N, x, y, dy, in_deriv=dx0)
        torch.cuda.synchronize()
        assert rel(dx0.cpu().numpy().astype(np.float64), dx_r) > 0.1
        c.close()
