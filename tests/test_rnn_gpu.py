"""RNN HIP kernels (cuDNN-shaped ABI, include/kaldi_rnn.h) and the fp32 MFMA
GEMM (include/kaldi_cumatrix.h) vs the fp64 oracle.

Tolerances (north_star: RNN gradients within 1e-4 relative fp32): norm-wise
relative error <= 1e-5 on y, <= 1e-4 on dx and dw."""
import numpy as np
import pytest

import sketch_common as S
from conftest import rel_err

pytestmark = pytest.mark.gpu


def _mk(kctc, gpu, mode, T, N, D, H, layers, bidir, seed, wscale=0.15, prec=None):
    import torch
    rng = np.random.default_rng(seed)
    r = kctc.Rnn(mode, D, H, layers, bidir)
    if prec is not None:  # part of the descriptor: before the size queries (kaldi_rnn.h)
        r.set_precision(prec)
    P = r.num_params
    w = (rng.standard_normal(P) * wscale).astype(np.float32)
    x = rng.standard_normal((T, N, D)).astype(np.float32)
    dy = rng.standard_normal((T, N, r.dirs * H)).astype(np.float32)
    ws_b, res_b = r.sizes(T, N)
    t = lambda a: torch.from_numpy(a).to(gpu)
    bufs = dict(w=t(w), x=t(x), dy=t(dy), y=torch.empty((T, N, r.dirs * H), device=gpu),
                dx=torch.empty((T, N, D), device=gpu), dw=torch.zeros(P, device=gpu),
                ws=torch.empty(ws_b, dtype=torch.uint8, device=gpu),
                res=torch.empty(res_b, dtype=torch.uint8, device=gpu))
    return r, (w, x, dy), bufs


def _run_gpu(r, b):
    import torch
    r.forward_training(b["x"], b["w"], b["y"], b["ws"], b["res"])
    r.backward_data(b["y"], b["dy"], b["w"], b["dx"], b["ws"], b["res"])
    r.backward_weights(b["x"], b["y"], b["dw"], b["ws"], b["res"])
    torch.cuda.synchronize()
    assert r.device_status() == 0
    return b["y"].cpu().numpy(), b["dx"].cpu().numpy(), b["dw"].cpu().numpy()


CASES = [
    # (mode, T, N, D, H, layers, bidir)
    (2, 23, 5, 24, 64, 1, True),     # LSTM, the recipe's component shape in miniature
    (2, 17, 3, 40, 64, 1, False),
    (2, 11, 4, 16, 32, 2, True),     # stacked (num-layers 2)
    (3, 19, 6, 20, 64, 1, True),     # GRU
    (3, 9, 2, 8, 48, 2, False),
    (0, 15, 4, 12, 32, 1, True),     # RELU
    (1, 15, 4, 12, 32, 1, True),     # TANH
    (2, 9, 40, 32, 64, 1, True),     # N > 16: several MFMA row tiles
    (2, 40, 16, 256, 512, 1, True),  # BLSTM-512 width (U=8 / U=16 partitions)
    # v6 (split-fp16 MFMA) shapes: H in {256, 320, 512}, N <= 16, LSTM and GRU
    (3, 21, 7, 64, 256, 1, True),    # GRU H=256, padded rows
    (2, 16, 5, 48, 320, 1, False),   # uni LSTM H=320 (the recipe's cell dim)
    (3, 12, 16, 40, 512, 2, True),   # stacked BGRU-512
    (2, 30, 1, 40, 256, 1, True),    # a single utterance
    # v6 row groups (N > 16: independent recurrences per 16 sequences)
    (2, 24, 64, 40, 512, 1, True),   # configs[2] width: 4 groups, U=32 on 512-thread workgroups
    (2, 18, 32, 64, 512, 1, True),   # 2 groups, U=16
    (3, 20, 33, 48, 256, 1, True),   # 3 groups, ragged last group (1 row)
    (3, 15, 45, 24, 512, 2, True),   # stacked, 3 groups
    (2, 14, 20, 16, 256, 1, False),  # uni, 2 groups
    # H = 1024 (configs[4] width)
    (3, 12, 8, 40, 1024, 1, True),   # one group, U=16
    (3, 10, 32, 40, 1024, 1, True),  # 2 groups, U=32 on 512-thread workgroups
]


@pytest.mark.parametrize("case", CASES, ids=[f"m{c[0]}_T{c[1]}_N{c[2]}_D{c[3]}_H{c[4]}_L{c[5]}_{'bi' if c[6] else 'uni'}"
                                             for c in CASES])
def test_rnn_matches_oracle(kctc, gpu, oracle, case):
    mode, T, N, D, H, layers, bidir = case
    r, (w, x, dy), b = _mk(kctc, gpu, mode, T, N, D, H, layers, bidir, seed=sum(case))
    assert r.num_params == oracle.params_size(mode, D, H, layers, r.dirs)
    y, dx, dw = _run_gpu(r, b)
    ry, res = oracle.rnn_forward(mode, x.astype(np.float64), w.astype(np.float64), H, layers, r.dirs)
    rdx, rdw = oracle.rnn_backward(mode, x.astype(np.float64), w.astype(np.float64), ry,
                                   dy.astype(np.float64), res, H, layers, r.dirs)
    assert rel_err(y, ry) < 1e-5
    assert rel_err(dx, rdx) < 1e-4
    assert rel_err(dw, rdw) < 1e-4
    # per-region check of dW (W, R, biases of every pseudo-layer)
    nlin = 2 * (4 if mode == 2 else 3 if mode == 3 else 1)
    for pl in range(layers * r.dirs):
        for lin in range(nlin):
            for isb in (0, 1):
                off, (h, c) = r.lin_offset(pl, lin, isb)
                sl = slice(off, off + h * c)
                assert rel_err(dw[sl], rdw[sl]) < 2e-4, (pl, lin, isb)


GS8_CASES = [
    # KCTC_REC_GS=8: a batch of 9..32 sequences runs as groups of 8 (side by side)
    (2, 24, 16, 40, 512, 1, True),   # configs[1] width: 2 groups of 8, U=16 on 512-thread workgroups
    (3, 20, 13, 48, 256, 1, True),   # ragged last group (5 rows)
    (2, 14, 12, 16, 256, 2, False),  # stacked uni
    (2, 12, 30, 40, 512, 1, True),   # 4 groups (the last one 6 rows), U=32
]


@pytest.mark.parametrize("case", GS8_CASES, ids=[f"m{c[0]}_T{c[1]}_N{c[2]}_H{c[4]}_L{c[5]}" for c in GS8_CASES])
def test_rnn_group8_matches_oracle(kctc, gpu, oracle, monkeypatch, case):
    """Row groups of 8 sequences (rows n0..n0+7 of each group's 16-row MFMA
    tile live, the other rows neither stored nor loaded) against the oracle."""
    monkeypatch.setenv("KCTC_REC_GS", "8")
    test_rnn_matches_oracle(kctc, gpu, oracle, case)


BF16_CASES = [
    # (mode, T, N, D, H, layers, bidir): configs[4] shapes in miniature
    (3, 20, 32, 64, 1024, 1, True),   # BGRU-1024, 2 row groups, U=32
    (3, 16, 8, 40, 1024, 1, True),    # one group, U=16
    (2, 18, 20, 48, 512, 1, True),    # BLSTM-512 in bf16
    (3, 12, 5, 32, 256, 2, False),    # stacked uni GRU
]
# bf16 operands (8 significant bits, relative rounding 2^-9) with fp32
# accumulation, against the fp64 oracle: norm-wise relative error bounds of
# the error model in sketch_common.bf16_tol (3 sigma over the chained stages)


@pytest.mark.parametrize("case", BF16_CASES, ids=[f"m{c[0]}_T{c[1]}_N{c[2]}_D{c[3]}_H{c[4]}_L{c[5]}" for c in BF16_CASES])
def test_rnn_bf16_matches_oracle(kctc, gpu, oracle, case):
    """krnnSetPrecision(KRNN_PREC_BF16): bf16 recurrences and gate GEMMs."""
    mode, T, N, D, H, layers, bidir = case
    r, (w, x, dy), b = _mk(kctc, gpu, mode, T, N, D, H, layers, bidir, seed=sum(case) + 1, wscale=0.05,
                           prec="bf16")
    y, dx, dw = _run_gpu(r, b)
    ry, res = oracle.rnn_forward(mode, x.astype(np.float64), w.astype(np.float64), H, layers, r.dirs)
    rdx, rdw = oracle.rnn_backward(mode, x.astype(np.float64), w.astype(np.float64), ry,
                                   dy.astype(np.float64), res, H, layers, r.dirs)
    errs = {"y": rel_err(y, ry), "dx": rel_err(dx, rdx), "dw": rel_err(dw, rdw)}
    print(case, {k: f"{v:.2e}" for k, v in errs.items()})
    for k, e in errs.items():
        assert e < S.bf16_tol(S.layer_stages(k, layers)), (k, e)
    # and it is the bf16 path: the fp32-class result is far closer
    r2, _, b2 = _mk(kctc, gpu, mode, T, N, D, H, layers, bidir, seed=sum(case) + 1, wscale=0.05)
    y2, _, _ = _run_gpu(r2, b2)
    assert rel_err(y2, ry) < 1e-5 < errs["y"]


def test_gemm_x3_rarely_active_columns(kctc, gpu):
    """dW-shaped split-fp16 GEMM (C = A^T B over K frames) whose A columns are
    "rarely active" gate units: a few frames O(1), the rest down to 1e-9 (a
    saturated sigmoid's derivative), so an output element can be dominated by
    terms far below the column maximum the power-of-two scale is taken from
    (their lo parts fall into fp16 subnormals).  Element-wise against fp64,
    normalised by the element's own sum of |terms| -- the bound an fp32 sgemm
    is held to -- and next to numpy's fp32 sgemm on the same operands."""
    import torch
    rng = np.random.default_rng(5)
    K, M, N = 6000, 192, 96
    A = rng.standard_normal((K, M)).astype(np.float32)
    act = rng.uniform(size=(K, M)) < np.array([1.0, 0.1, 0.01, 0.001])[np.arange(M) % 4]
    A = np.where(act, A, A * (10.0 ** rng.uniform(-9, -3, (K, M)))).astype(np.float32)
    B = np.tanh(rng.standard_normal((K, N))).astype(np.float32)   # h in (-1, 1)
    B[rng.uniform(size=(K, N)) < 0.3] = 0.0                       # units off at many frames
    C = torch.zeros((M, N), dtype=torch.float32, device=gpu)
    kctc.add_mat_mat_x3(C, torch.from_numpy(A).to(gpu), torch.from_numpy(B).to(gpu), True, False,
                        alpha=1.0, beta=0.0)
    torch.cuda.synchronize()
    ref = A.T.astype(np.float64) @ B.astype(np.float64)
    den = np.abs(A.T).astype(np.float64) @ np.abs(B).astype(np.float64) + 1e-300
    e_x3 = np.abs(C.cpu().numpy().astype(np.float64) - ref) / den
    e_f32 = np.abs((A.T @ B).astype(np.float64) - ref) / den
    print(f"max element error / sum|terms|: x3 {e_x3.max():.2e}, fp32 sgemm {e_f32.max():.2e}")
    # measured: x3 2.3e-6, numpy fp32 sgemm 1.2e-6 (both far inside the 1e-4 bar)
    assert e_x3.max() < 1e-5
    assert e_x3.max() < 5 * max(e_f32.max(), 6e-8)


def test_rnn_golden_layout(kctc, gpu):
    """The torch-fp64 golden fixture through the HIP path (cuDNN layout)."""
    import torch
    from conftest import golden
    g = golden("rnn_lstm_bi_h32")
    mode, H, layers, dirs = int(g["mode"]), int(g["H"]), int(g["layers"]), int(g["dirs"])
    T, N, D = g["x"].shape
    r = kctc.Rnn(mode, D, H, layers, dirs == 2)
    ws_b, res_b = r.sizes(T, N)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    b = dict(w=t(g["w"]), x=t(g["x"]), dy=t(g["dy"]), y=torch.empty((T, N, dirs * H), device=gpu),
             dx=torch.empty((T, N, D), device=gpu), dw=torch.zeros(g["w"].size, device=gpu),
             ws=torch.empty(ws_b, dtype=torch.uint8, device=gpu),
             res=torch.empty(res_b, dtype=torch.uint8, device=gpu))
    y, dx, dw = _run_gpu(r, b)
    assert rel_err(y, g["y"]) < 1e-5
    assert rel_err(dx, g["dx"]) < 1e-4
    assert rel_err(dw, g["dw"]) < 1e-4


def test_rnn_weights_accumulate_and_inference(kctc, gpu, oracle):
    import torch
    r, (w, x, dy), b = _mk(kctc, gpu, 2, 13, 4, 16, 32, 1, True, seed=3)
    _, _, dw1 = _run_gpu(r, b)
    # second BackwardWeights accumulates (cudnnRNNBackwardWeights semantics)
    r.backward_weights(b["x"], b["y"], b["dw"], b["ws"], b["res"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(b["dw"].cpu().numpy(), 2 * dw1, rtol=1e-5, atol=1e-6)
    y_inf = torch.empty_like(b["y"])
    ws = torch.empty(r.sizes(13, 4)[0], dtype=torch.uint8, device=gpu)
    r.forward_inference(b["x"], b["w"], y_inf, ws)
    torch.cuda.synchronize()
    assert torch.equal(y_inf, b["y"])


def test_rnn_full_size_properties(kctc, gpu):
    """configs[1] layer 2-5 shape (T=2000, N=16, D=1024, H=512, bidir): too big
    for the fp64 oracle in test time, so check size-independent properties:
    bitwise determinism, finite outputs, no sentinel left in the exchange."""
    import torch
    T, N, D, H = 2000, 16, 1024, 512
    r = kctc.Rnn(2, D, H, 1, True)
    g = torch.Generator(device=gpu).manual_seed(0)
    w = torch.randn(r.num_params, device=gpu, generator=g) * 0.02
    x = torch.randn((T, N, D), device=gpu, generator=g)
    dy = torch.randn((T, N, 2 * H), device=gpu, generator=g)
    ws_b, res_b = r.sizes(T, N)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=gpu)
    res = torch.empty(res_b, dtype=torch.uint8, device=gpu)
    outs = []
    for _ in range(2):
        y = torch.empty((T, N, 2 * H), device=gpu)
        dx = torch.empty((T, N, D), device=gpu)
        dw = torch.zeros(r.num_params, device=gpu)
        r.forward_training(x, w, y, ws, res)
        r.backward_data(y, dy, w, dx, ws, res)
        r.backward_weights(x, y, dw, ws, res)
        torch.cuda.synchronize()
        assert r.device_status() == 0
        outs.append((y, dx, dw))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
        assert torch.isfinite(a).all()
    # forward direction at t=0 depends only on x[0]: compare with a T=1 run
    y1 = torch.empty((1, N, 2 * H), device=gpu)
    ws1 = torch.empty(r.sizes(1, N)[0], dtype=torch.uint8, device=gpu)
    res1 = torch.empty(r.sizes(1, N)[1], dtype=torch.uint8, device=gpu)
    r.forward_training(x[:1].contiguous(), w, y1, ws1, res1)
    torch.cuda.synchronize()
    assert torch.allclose(y1[0, :, :H], outs[0][0][0, :, :H], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("ta,tb,M,N,K", [(0, 0, 77, 41, 40), (0, 1, 300, 130, 257), (1, 0, 64, 96, 1000),
                                         (1, 1, 33, 17, 9), (0, 1, 1024, 1024, 1024)])
def test_gemm_matches_numpy(kctc, gpu, ta, tb, M, N, K):
    import torch
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    C = torch.from_numpy(C0).to(gpu)
    kctc.add_mat_mat(C, torch.from_numpy(A).to(gpu), torch.from_numpy(B).to(gpu), bool(ta), bool(tb),
                     alpha=0.5, beta=-1.5)
    torch.cuda.synchronize()
    ref = 0.5 * ((A.T if ta else A).astype(np.float64) @ (B.T if tb else B).astype(np.float64)) - 1.5 * C0
    assert rel_err(C.cpu().numpy(), ref) < 1e-6


@pytest.mark.parametrize("ta,tb,M,N,K,beta", [(0, 0, 77, 41, 40, 0.0), (0, 1, 300, 130, 257, 0.0),
                                              (1, 0, 64, 96, 1000, 0.0), (1, 1, 33, 17, 9, 0.0),
                                              (0, 1, 1024, 1024, 1024, 0.0), (1, 0, 512, 256, 4000, 0.0),
                                              # 256 x 256 tiles with ragged edges in both dimensions
                                              # (16-B row pieces where ldc allows, element stores otherwise)
                                              (0, 1, 300, 260, 257, 0.0), (1, 0, 700, 450, 3000, 0.0),
                                              (0, 1, 520, 300, 700, -1.5), (0, 0, 700, 451, 300, 0.75)])
def test_gemm_x3_matches_numpy(kctc, gpu, ta, tb, M, N, K, beta):
    """Split-fp16 GEMM: fp32-class accuracy, also for rows / columns whose
    magnitudes differ by many orders (per-row / per-column power-of-two scaling)."""
    import torch
    rng = np.random.default_rng(M * 7 + N + K)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    # op(A) rows and op(B) columns spanning 1e-12 .. 1e6
    ra = (10.0 ** rng.uniform(-12, 6, M)).astype(np.float32)
    cb = (10.0 ** rng.uniform(-12, 6, N)).astype(np.float32)
    A = A * (ra[None, :] if ta else ra[:, None])
    B = B * (cb[:, None] if tb else cb[None, :])
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    C = torch.from_numpy(C0).to(gpu)
    kctc.add_mat_mat_x3(C, torch.from_numpy(A).to(gpu), torch.from_numpy(B).to(gpu), bool(ta), bool(tb),
                        alpha=0.5, beta=beta)
    torch.cuda.synchronize()
    ref = 0.5 * ((A.T if ta else A).astype(np.float64) @ (B.T if tb else B).astype(np.float64)) + beta * C0
    out = C.cpu().numpy().astype(np.float64)
    # element-wise, relative to the scale of the row of op(A) times the column of op(B)
    scale = np.abs(A.T if ta else A).max(axis=1)[:, None] * np.abs(B.T if tb else B).max(axis=0)[None, :] * K
    scale = scale + 4 * np.abs(beta * C0)
    assert np.max(np.abs(out - ref) / scale) < 2e-7
    assert rel_err(out, ref) < 1e-6
