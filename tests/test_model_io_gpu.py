"""Model I/O: nnet2-ctc model files in Kaldi binary and text
mode -- CtcTransitionModel (kept opaque) + AmNnet (Nnet + priors) with the
<CuDNNRecurrentComponent> <FilterParams> layout -- through kctc_am_nnet_* /
kctc_nnet_write_kaldi / kctc_nnet_read.

Oracle: an independent Python writer of the Kaldi binary token stream
(base/io-funcs-inl.h WriteBasicType / WriteIntegerVector, kaldi-vector.cc /
kaldi-matrix.cc Write, nnet-nnet.cc:170-183, am-nnet.cc:31-37 and the
component Write functions nnet-cudnn-component.cc:698-721, 814-837,
nnet-component.cc:1260-1274, 2822-2831).  The reference tree holds no model
file, so byte parity is against this restatement ("parity unpinned" against a
Kaldi binary).  A model the writer produced must load with the same
parameters and be written back byte for byte.
"""
import struct

import numpy as np
import pytest

import oracle_lib as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


def tok(t):
    return t.encode() + b" "


def i32(v):
    return b"\x04" + struct.pack("<i", v)


def f32(v):
    return b"\x04" + struct.pack("<f", v)


def bl(b):
    return b"T" if b else b"F"


def fvec(a):
    a = np.ascontiguousarray(a, dtype="<f4")
    return tok("FV") + i32(a.size) + a.tobytes()


def fmat(m):
    m = np.ascontiguousarray(m, dtype="<f4")
    return tok("FM") + i32(m.shape[0]) + i32(m.shape[1]) + m.tobytes()


def ivec(v):
    return b"\x04" + struct.pack("<i", len(v)) + np.asarray(v, dtype="<i4").tobytes()


def splice(D):
    return (tok("<SpliceComponent>") + tok("<InputDim>") + i32(D) + tok("<Context>") + ivec([0]) +
            tok("<ConstComponentDim>") + i32(0) + tok("</SpliceComponent>"))


def rnn(lr, D, H, mode, bidir, params, max_seq=2000, clip=5.0):
    return (tok("<CuDNNRecurrentComponent>") + tok("<LearningRate>") + f32(lr) + tok("<IsGradient>") + bl(False) +
            tok("<ClipGradient>") + f32(clip) + tok("<InputDim>") + i32(D) + tok("<HiddenDim>") + i32(H) +
            tok("<NumLayers>") + i32(1) + tok("<Bidirectional>") + bl(bidir) + tok("<RNNMode>") + i32(mode) +
            tok("<MaxSeqLength>") + i32(max_seq) + tok("<FilterParams>") + fvec(params) +
            tok("</CuDNNRecurrentComponent>"))


def clipgrad(dim, counters=(5, 100, 0, 3)):
    return (tok("<ClipGradientComponent>") + tok("<Dim>") + i32(dim) + tok("<ClippingThreshold>") + f32(30.0) +
            tok("<NormBasedClipping>") + bl(True) + tok("<SelfRepairClippedProportionThreshold>") + f32(0.01) +
            tok("<SelfRepairTarget>") + f32(0.0) + tok("<SelfRepairScale>") + f32(1.0) +
            tok("<NumElementsClipped>") + i32(counters[0]) + tok("<NumElementsProcessed>") + i32(counters[1]) +
            tok("<NumSelfRepaired>") + i32(counters[2]) + tok("<NumBackpropped>") + i32(counters[3]) +
            tok("</ClipGradientComponent>"))


def affine(lr, W, b):
    return (tok("<AffineComponent>") + tok("<LearningRate>") + f32(lr) + tok("<LinearParams>") + fmat(W) +
            tok("<BiasParams>") + fvec(b) + tok("<IsGradient>") + bl(False) + tok("</AffineComponent>"))


def nnet(components):
    return (tok("<Nnet>") + tok("<NumComponents>") + i32(len(components)) + tok("<Components>") +
            b"".join(components) + tok("</Components>") + tok("</Nnet>"))


TRANS = (tok("<TransitionModel>") + tok("<Topology>") + b"\x04\x07\x00\x00\x00" + bytes(range(256)) +
         tok("</Topology>") + tok("<LogProbs>") + fvec(np.linspace(-3, 0, 11)) + tok("</LogProbs>") +
         tok("</TransitionModel>"))


def build_model(rng, D=16, H=32, A=9, mode=2):
    P = O.params_size(mode, D, H, 1, 2)
    p1 = rng.standard_normal(P).astype(np.float32) * 0.02
    P2 = O.params_size(mode, 2 * H, H, 1, 2)
    p2 = rng.standard_normal(P2).astype(np.float32) * 0.02
    W = rng.standard_normal((A, 2 * H)).astype(np.float32)
    b = rng.standard_normal(A).astype(np.float32)
    comps = [splice(D), rnn(5e-4, D, H, mode, True, p1), clipgrad(2 * H),
             rnn(5e-4, 2 * H, H, mode, True, p2, max_seq=1234), clipgrad(2 * H, (0, 0, 0, 0)), affine(2.5e-4, W, b)]
    params = [None, p1, None, p2, None, np.concatenate([W.ravel(), b])]
    return comps, params


@pytest.mark.parametrize("with_trans,with_priors", [(True, True), (False, True), (True, False)])
def test_am_model_binary_loads_and_writes_back_byte_identical(kctc, gpu, tmp_path, with_trans, with_priors):
    rng = np.random.default_rng(4)
    comps, params = build_model(rng)
    priors = rng.random(9).astype(np.float32) if with_priors else np.zeros(0, np.float32)
    blob = b"\0B" + (TRANS if with_trans else b"") + nnet(comps) + fvec(priors)
    src = tmp_path / "final.mdl"
    src.write_bytes(blob)
    net = kctc.Nnet.read_am(src)
    assert net.num_components == 6
    for c, p in enumerate(params):
        if p is not None:
            np.testing.assert_array_equal(net.get_params(c), p)
    np.testing.assert_array_equal(net.priors, priors)
    out = tmp_path / "out.mdl"
    net.write_am(out, binary=True)
    assert out.read_bytes() == blob
    net.close()


def test_nnet_binary_matches_restatement_and_text_round_trip(kctc, gpu, tmp_path):
    """Nnet::Write binary of a created network == the restatement built from its
    own parameters; binary round trips are exact, text ones keep the 7
    significant digits of Kaldi's text streams (InitKaldiOutputStream,
    base/io-funcs-inl.h:296-302) and are a fixed point after one pass."""
    D, H, A = 16, 32, 9
    net = kctc.Nnet(kctc.recipe_config(num_rnn=2, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4), seed=7)
    pb, pt = tmp_path / "n.bin", tmp_path / "n.txt"
    net.write(pb, binary=True)
    net.write(pt, binary=False)
    data = pb.read_bytes()
    assert data.startswith(b"\0B<Nnet> <NumComponents> \x04")
    # every parameter vector appears verbatim, in component order
    pos = 0
    for c in range(net.num_components):
        if net.num_params(c):
            raw = net.get_params(c).astype("<f4").tobytes()
            if c == net.num_components - 1:  # affine: W then b, each behind its header
                W = raw[:4 * A * 2 * H]
                i = data.index(tok("FM") + i32(A) + i32(2 * H) + W, pos)
            else:
                i = data.index(tok("FV") + i32(len(raw) // 4) + raw, pos)
            pos = i + 1
    n2 = kctc.Nnet.read(pb)
    for c in range(net.num_components):
        if net.num_params(c):
            np.testing.assert_array_equal(n2.get_params(c), net.get_params(c))
    p2 = tmp_path / "again.bin"
    n2.write(p2, binary=True)
    assert p2.read_bytes() == data
    n2.close()
    n3 = kctc.Nnet.read(pt)
    for c in range(net.num_components):
        if net.num_params(c):
            np.testing.assert_allclose(n3.get_params(c), net.get_params(c), rtol=6e-7, atol=1e-30)
    p3 = tmp_path / "again.txt"
    n3.write(p3, binary=False)
    assert p3.read_bytes() == pt.read_bytes()
    n3.close()


def test_am_model_text_mode_and_priors(kctc, gpu, tmp_path):
    rng = np.random.default_rng(5)
    comps, params = build_model(rng, mode=3)  # GRU
    src = tmp_path / "m.mdl"
    src.write_bytes(b"\0B" + nnet(comps) + fvec(np.zeros(0, np.float32)))
    net = kctc.Nnet.read_am(src)
    assert net.priors.size == 0
    with pytest.raises(RuntimeError):
        net.set_priors(np.ones(10))  # > number of pdfs (am-nnet.cc:46-47)
    net.set_priors([0.5, 0.25])  # zero-extended (:49-54)
    np.testing.assert_array_equal(net.priors, np.array([0.5, 0.25] + [0] * 7, np.float32))
    txt = tmp_path / "m.txt"
    net.write_am(txt, binary=False)
    t = txt.read_text()
    assert t.startswith("<Nnet> <NumComponents> 6") and "<CuDNNRecurrentComponent>" in t
    net2 = kctc.Nnet.read_am(txt)
    for c, p in enumerate(params):
        if p is not None:  # text: 7 significant digits
            np.testing.assert_allclose(net2.get_params(c), p, rtol=6e-7, atol=1e-30)
    np.testing.assert_array_equal(net2.priors, net.priors)
    back = tmp_path / "back.txt"
    net2.write_am(back, binary=False)
    assert back.read_bytes() == txt.read_bytes()
    pri = np.array([0.5, 0.25] + [0] * 7, np.float32)
    # a text transition model is kept with its trailing newline
    # (transition-model.cc:316-317): text write-back is byte-identical
    ttrans = (b"<TransitionModel> \n<Topology> \n<TopologyEntry> \n</TopologyEntry> \n</Topology> \n"
              b"<Triples> 0 \n</Triples> \n<LogProbs> \n [ ]\n</LogProbs> \n</TransitionModel> \n")
    src3 = tmp_path / "tt.mdl"
    src3.write_bytes(ttrans + txt.read_bytes())
    n4 = kctc.Nnet.read_am(src3)
    out4 = tmp_path / "tt_out.mdl"
    n4.write_am(out4, binary=False)
    assert out4.read_bytes() == src3.read_bytes()
    n4.close()
    # a binary transition model cannot be re-emitted in text mode
    src2 = tmp_path / "t.mdl"
    src2.write_bytes(b"\0B" + TRANS + nnet(comps) + fvec(pri))
    n3 = kctc.Nnet.read_am(src2)
    with pytest.raises(RuntimeError):
        n3.write_am(tmp_path / "x.txt", binary=False)
    for n in (net, net2, n3):
        n.close()


def test_old_component_forms_are_read(kctc, gpu, tmp_path):
    """Back-compatibility branches of the reference readers: Splice
    <LeftContext>/<RightContext>, ClipGradient without the self-repair fields,
    Affine with <AvgInput>."""
    rng = np.random.default_rng(6)
    comps, params = build_model(rng)
    comps[0] = (tok("<SpliceComponent>") + tok("<InputDim>") + i32(16) + tok("<LeftContext>") + i32(0) +
                tok("<RightContext>") + i32(0) + tok("<ConstComponentDim>") + i32(0) + tok("</SpliceComponent>"))
    comps[2] = (tok("<ClipGradientComponent>") + tok("<Dim>") + i32(64) + tok("<ClippingThreshold>") + f32(30.0) +
                tok("<NormBasedClipping>") + bl(True) + tok("<NumElementsClipped>") + i32(1) +
                tok("<NumElementsProcessed>") + i32(2) + tok("</ClipGradientComponent>"))
    W, b = params[5][:9 * 64].reshape(9, 64), params[5][9 * 64:]
    comps[5] = (tok("<AffineComponent>") + tok("<LearningRate>") + f32(1e-3) + tok("<LinearParams>") + fmat(W) +
                tok("<BiasParams>") + fvec(b) + tok("<AvgInput>") + fvec(np.ones(64)) + tok("<AvgInputCount>") +
                f32(3.0) + tok("<IsGradient>") + bl(False) + tok("</AffineComponent>"))
    p = tmp_path / "old.mdl"
    p.write_bytes(b"\0B" + nnet(comps))
    net = kctc.Nnet.read(p)
    np.testing.assert_array_equal(net.get_params(5), params[5])
    info = net.info(2)
    assert "ClipGradient" in info
    net.close()


def test_bad_models_are_refused(kctc, gpu, tmp_path):
    """Reader checks (nnet-component.cc SpliceComponent / nnet-cudnn-component.cc
    InitFromString, nnet-nnet.cc Check): a spliced model (context != {0}: this
    path aliases the input), an out-of-range <RNNMode>, a dimension mismatch
    between components -- clean errors, not out-of-bounds device accesses."""
    rng = np.random.default_rng(8)
    comps, params = build_model(rng)
    bad = []
    c = list(comps)
    c[0] = (tok("<SpliceComponent>") + tok("<InputDim>") + i32(16) + tok("<LeftContext>") + i32(1) +
            tok("<RightContext>") + i32(1) + tok("<ConstComponentDim>") + i32(0) + tok("</SpliceComponent>"))
    bad.append(c)
    c = list(comps)
    c[1] = rnn(5e-4, 16, 32, 5, True, params[1])
    bad.append(c)
    c = list(comps)
    c[2] = clipgrad(48)  # RNN output 64 -> ClipGradient 48
    bad.append(c)
    for i, cs in enumerate(bad):
        p = tmp_path / f"bad{i}.mdl"
        p.write_bytes(b"\0B" + nnet(cs))
        with pytest.raises(RuntimeError):
            kctc.Nnet.read(p)


def test_affine_is_gradient_round_trips(kctc, gpu, tmp_path):
    rng = np.random.default_rng(9)
    comps, params = build_model(rng)
    W, b = params[5][:9 * 64].reshape(9, 64), params[5][9 * 64:]
    comps[5] = (tok("<AffineComponent>") + tok("<LearningRate>") + f32(1e-3) + tok("<LinearParams>") + fmat(W) +
                tok("<BiasParams>") + fvec(b) + tok("<IsGradient>") + bl(True) + tok("</AffineComponent>"))
    blob = b"\0B" + nnet(comps)
    p = tmp_path / "g.mdl"
    p.write_bytes(blob)
    net = kctc.Nnet.read(p)
    out = tmp_path / "g_out.mdl"
    net.write(out, binary=True)
    assert out.read_bytes() == blob
    net.close()
