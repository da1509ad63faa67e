"""Pin the CPU oracle against the committed golden fixtures (torch fp64).

The reference holds no golden vectors for this path and its
arithmetic libraries are absent (§8c), so these fixtures -- produced by an
independent implementation of the same published equations -- are what pins
the oracle.  Tolerances: 1e-9 relative in fp64 (same math, different order).
"""
import numpy as np
import pytest

from conftest import golden, golden_names, rel_err


@pytest.mark.parametrize("name", golden_names("ctc_"))
def test_ctc_f64_matches_golden(oracle, name):
    g = golden(name)
    costs, grads = oracle.ctc(g["acts"].astype(np.float64), g["flat_labels"], g["label_lengths"],
                              g["input_lengths"])
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-9, atol=1e-9)
    assert rel_err(grads, g["grads"]) < 1e-9
    # padding rows carry zero gradient
    for n, tn in enumerate(g["input_lengths"]):
        assert np.all(grads[tn:, n, :] == 0)


@pytest.mark.parametrize("name", golden_names("ctc_"))
def test_ctc_f32_port_close(oracle, name):
    g = golden(name)
    costs, grads = oracle.ctc(g["acts"], g["flat_labels"], g["label_lengths"], g["input_lengths"])
    np.testing.assert_allclose(costs, g["costs"], rtol=1e-4, atol=1e-4)
    # plain fp32 log-space alpha/beta (warp-ctc's own arithmetic) loses ~1e-3
    # relative on gamma = exp(alpha+beta-logp) once |alpha| ~ 1e3: that is why
    # the HIP kernel carries per-frame offsets in fp64 (CTC kernel).
    assert rel_err(grads, g["grads"]) < 5e-3


def test_ctc_infeasible_is_zero(oracle):
    # L + repeats > T: warp-ctc CPU returns cost 0 and leaves the gradient alone
    acts = np.random.default_rng(0).standard_normal((3, 1, 5))
    costs, grads = oracle.ctc(acts, np.array([1, 1, 2], np.int32), np.array([3], np.int32),
                              np.array([3], np.int32))
    assert costs[0] == 0 and np.all(grads == 0)


def test_ctc_gradient_sums_to_zero(oracle):
    # sum_a (y - gamma) = 1 - 1 on every real frame
    g = golden("ctc_a41")
    _, grads = oracle.ctc(g["acts"].astype(np.float64), g["flat_labels"], g["label_lengths"],
                          g["input_lengths"])
    np.testing.assert_allclose(grads.sum(-1), 0, atol=1e-12)


@pytest.mark.parametrize("name", golden_names("rnn_"))
def test_rnn_f64_matches_golden(oracle, name):
    g = golden(name)
    mode, H, layers, dirs = int(g["mode"]), int(g["H"]), int(g["layers"]), int(g["dirs"])
    T, N, D = g["x"].shape
    assert g["w"].size == oracle.params_size(mode, D, H, layers, dirs)
    x = g["x"].astype(np.float64)
    w = g["w"].astype(np.float64)
    y, res = oracle.rnn_forward(mode, x, w, H, layers, dirs)
    assert rel_err(y, g["y"]) < 1e-10
    dx, dw = oracle.rnn_backward(mode, x, w, y, g["dy"].astype(np.float64), res, H, layers, dirs)
    assert rel_err(dx, g["dx"]) < 1e-10
    assert rel_err(dw, g["dw"]) < 1e-10


@pytest.mark.parametrize("name", ["rnn_lstm_bi", "rnn_gru_bi", "rnn_tanh_bi"])
def test_rnn_f32_port_close(oracle, name):
    g = golden(name)
    mode, H, layers, dirs = int(g["mode"]), int(g["H"]), int(g["layers"]), int(g["dirs"])
    y, res = oracle.rnn_forward(mode, g["x"], g["w"], H, layers, dirs)
    assert rel_err(y, g["y"]) < 1e-5
    dx, dw = oracle.rnn_backward(mode, g["x"], g["w"], y, g["dy"], res, H, layers, dirs)
    assert rel_err(dx, g["dx"]) < 1e-4
    assert rel_err(dw, g["dw"]) < 1e-4


def test_lin_layer_offsets_tile_the_buffer(oracle):
    # every (pseudo-layer, lin id, matrix|bias) region is disjoint and covers P
    for mode, nlin in ((0, 2), (1, 2), (2, 8), (3, 6)):
        D, H, layers, dirs = 7, 5, 2, 2
        P = oracle.params_size(mode, D, H, layers, dirs)
        cover = np.zeros(P, np.int32)
        for pl in range(layers * dirs):
            din = D if pl // dirs == 0 else dirs * H
            for lin in range(nlin):
                off = oracle.lin_offset(mode, D, H, layers, dirs, pl, lin, 0)
                sz = H * (din if lin < nlin // 2 else H)
                cover[off:off + sz] += 1
                off = oracle.lin_offset(mode, D, H, layers, dirs, pl, lin, 1)
                cover[off:off + H] += 1
        assert np.all(cover == 1)


def test_cudnn_param_count_blstm512(oracle):
    # P = 2,269,184 (layer 1) and 6,299,648 (layers 2-5)
    assert oracle.params_size(2, 40, 512, 1, 2) == 2269184
    assert oracle.params_size(2, 1024, 512, 1, 2) == 6299648
    assert oracle.params_size(3, 40, 1024, 1, 2) == 6549504
    assert oracle.params_size(3, 2048, 1024, 1, 2) == 18886656


def _cfg0_spec(oracle, g):
    s = oracle.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = 1, 2, int(g["H"]), 1, 1
    s.input_dim, s.num_targets = int(g["D"]), int(g["A"])
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, float(g["lr"]), float(g["lr"])
    return s


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_train_step_cfg0_matches_golden(oracle, dtype):
    g = golden("step_cfg0")
    spec = _cfg0_spec(oracle, g)
    w = g["w0"].astype(dtype).copy()
    Wa = g["Wa0"].astype(dtype).copy()
    ba = g["ba0"].astype(dtype).copy()
    tot, acc, wt = oracle.train_step(spec, [w], Wa, ba, g["feats"].astype(dtype), g["num_frames"],
                                     g["flat_labels"], g["label_lengths"],
                                     repair_draws=np.ones(1, np.float32))
    tol = 1e-9 if dtype == np.float64 else 1e-4
    np.testing.assert_allclose(tot, g["costs"].sum(), rtol=tol)
    assert wt == g["label_lengths"].sum()
    assert rel_err(w - g["w0"].astype(dtype), g["w_delta"]) < (1e-6 if dtype == np.float64 else 1e-3)
    assert rel_err(Wa - g["Wa0"].astype(dtype), g["Wa_delta"]) < (1e-6 if dtype == np.float64 else 1e-3)
    assert rel_err(ba - g["ba0"].astype(dtype), g["ba_delta"]) < (1e-6 if dtype == np.float64 else 1e-3)
    # accuracy matches the best path of the golden logits through the reference collapse rule
    ids = oracle.find_row_max_id(g["logits"].reshape(-1, int(g["A"])))
    acc_ref, _ = oracle.accuracy(ids, int(g["T"]), int(g["N"]), g["num_frames"], g["flat_labels"],
                                 g["label_lengths"])
    assert acc == acc_ref


def _find_row_max_id_lockstep(row):
    """Literal transcription of _find_row_max_id (src/cudamatrix/cu-kernels.cu:
    2454-2500) for one row: 256 threads (CU1DBLOCK, cu-matrixdim.h:63), the
    strided scan, the __syncthreads() levels 128/64/32 and the warp levels
    16..1 (warpSize 32), every thread of a level reading before any writes."""
    B = 256
    smax = [np.float32(-1e20)] * B
    sidx = [-1] * B
    for t in range(B):
        for j in range(t, len(row), B):
            if row[j] > smax[t]:
                smax[t], sidx[t] = row[j], j
    w = B // 2
    while w >= 1:
        active = range(w) if w >= 32 else range(16)  # warp part: tid < warpSize / 2
        take = [(p, smax[p + w], sidx[p + w]) for p in active if smax[p + w] > smax[p]]
        for p, v, i in take:
            smax[p], sidx[p] = v, i
        w //= 2
    return sidx[0]


def test_find_row_max_id_gpu_tie_rule(oracle):
    """The reference's CTC path runs the GPU _find_row_max_id: ties resolve by
    its reduction tree, not to the first column (the CPU rule)."""
    m = np.full((4, 41), -3.0, np.float32)
    m[0, [1, 2]] = 7.0         # tree: 2 (CPU rule: 1)
    m[1, [0, 1]] = 7.0         # 0
    m[2, :] = -1e20            # nothing above -1e20: -1
    m[3, [5, 37]] = 2.0        # 37 sits in thread 37's slot; 5 wins through the tree
    got = oracle.find_row_max_id(m)
    assert got.tolist() == [_find_row_max_id_lockstep(r) for r in m]
    assert got[:3].tolist() == [2, 0, -1]
    assert oracle.find_row_max_id(m, cpu_rule=True)[:3].tolist() == [1, 0, 0]  # CPU floor is -1e21


@pytest.mark.parametrize("cols", [1, 5, 41, 64, 256, 257, 300, 700])
def test_find_row_max_id_matches_lockstep_kernel(oracle, cols):
    rng = np.random.default_rng(cols)
    m = rng.integers(-3, 3, size=(40, cols)).astype(np.float32)  # many ties
    m[0] = -1e20
    m[1] = np.nan
    m[2, ::2] = -np.inf
    m[3, :] = -2e20
    m[3, -1] = -9.9e19
    got = oracle.find_row_max_id(m)
    want = [_find_row_max_id_lockstep(r) for r in m]
    assert got.tolist() == want
    assert got[0] == -1 and got[1] == -1 and got[3] == cols - 1


def test_accuracy_collapse_keeps_first_frame(oracle):
    # hyp[0] is always kept even if blank (ctc-nnet-update.cc:291-303)
    T, N = 6, 1
    ids = np.array([0, 3, 3, 0, 4, 4], np.int32)
    acc, w = oracle.accuracy(ids, T, N, np.array([6], np.int32), np.array([3, 4], np.int32),
                             np.array([2], np.int32))
    # hyp = [0, 3, 4] vs ref [3, 4] -> 1 edit
    assert w == 2 and acc == 1
    assert oracle.lib().oracle_levenshtein(np.array([1, 2, 3], np.int32), 3,
                                           np.array([1, 3], np.int32), 2) == 1
