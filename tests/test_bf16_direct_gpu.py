"""bf16 recurrences write their dGates straight into the packed bf16 operands
of the dx / dW / dR GEMMs (rnn.hip bf16_direct, RecParams::dxr / dxt / et)
instead of fp32 rows that pack kernels convert afterwards.  The conversion is
the same round-to-nearest cast of the same fp32 values, so training is bit
identical to the packing path (KCTC_BF16_DIRECT=0), for GRU (separate DX and E
transposes) and LSTM (one), ragged frame counts whose packed rows end in a
zero tail (T*N not a multiple of 64), and groups of fewer than 16 rows
(KCTC_BF16_IO=0).  With the forward's output packed too (bf16_io: y rows and
columns from the recurrence, E^T written shifted by one step so that dR pairs
it with the unshifted y^T) the dR products are the same but sit N frames
further along the GEMM's K: its k-blocks group them differently, so the sums
round differently -- same to 1e-6 of the parameters after one step instead
of bit for bit."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _train(kctc, gpu, cfg, batch, direct, steps=2, io=False):
    import torch
    feats, nf, fl, ll, T, N = batch
    old = os.environ.get("KCTC_BF16_DIRECT")
    old_io = os.environ.get("KCTC_BF16_IO")
    os.environ["KCTC_BF16_DIRECT"] = "1" if direct else "0"
    os.environ["KCTC_BF16_IO"] = "1" if io else "0"
    try:
        net = kctc.Nnet(cfg, seed=3)
        net.set_precision("bf16")
        f = torch.from_numpy(feats).to(gpu)
        stats = [net.train_step(f, T, N, nf, fl, ll) for _ in range(steps)]
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.close()
    finally:
        for k, v in (("KCTC_BF16_DIRECT", old), ("KCTC_BF16_IO", old_io)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return stats, params


@pytest.mark.parametrize("mode,H,N,T", [(3, 1024, 32, 120), (3, 1024, 20, 77), (2, 512, 16, 90), (3, 512, 40, 61)])
def test_direct_packing_bit_identical(kctc, gpu, mode, H, N, T):
    D, A, R = 40, 41, 2
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                             max_seq_length=T, rnn_mode=mode)
    feats, nf, fl, ll = kctc.synth_minibatch(17 + N, T, N, D, A, 0.125)
    batch = (feats, nf, fl, ll, T, N)
    a = _train(kctc, gpu, cfg, batch, direct=False)
    b = _train(kctc, gpu, cfg, batch, direct=True)
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)
    # one step: the next one's bf16 casts of the updated weights turn a 1e-8
    # difference into whole bf16 ulps, so the runs drift apart (both equally
    # far from the fp64 oracle: test_train_step_bf16_matches_oracle)
    a = _train(kctc, gpu, cfg, batch, direct=False, steps=1)
    c = _train(kctc, gpu, cfg, batch, direct=True, io=True, steps=1)
    for sa, sc in zip(a[0], c[0]):
        np.testing.assert_allclose(np.asarray(sc, dtype=np.float64), np.asarray(sa, dtype=np.float64), rtol=1e-5)
    for x, y in zip(a[1], c[1]):
        np.testing.assert_allclose(y, x, rtol=0, atol=1e-6)
