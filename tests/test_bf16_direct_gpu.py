"""bf16 recurrences write their dGates straight into the packed bf16 operands
of the dx / dW / dR GEMMs (rnn.hip bf16_direct, RecParams::dxr / dxt / et)
instead of fp32 rows that pack kernels convert afterwards.  The conversion is
the same round-to-nearest cast of the same fp32 values, so training is bit
identical to the packing path (KCTC_BF16_DIRECT=0), for GRU (separate DX and E
transposes) and LSTM (one), ragged frame counts whose packed rows end in a
zero tail (T*N not a multiple of 64), and groups of fewer than 16 rows."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _train(kctc, gpu, cfg, batch, direct, steps=2):
    import torch
    feats, nf, fl, ll, T, N = batch
    old = os.environ.get("KCTC_BF16_DIRECT")
    os.environ["KCTC_BF16_DIRECT"] = "1" if direct else "0"
    try:
        net = kctc.Nnet(cfg, seed=3)
        net.set_precision("bf16")
        f = torch.from_numpy(feats).to(gpu)
        stats = [net.train_step(f, T, N, nf, fl, ll) for _ in range(steps)]
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.close()
    finally:
        if old is None:
            os.environ.pop("KCTC_BF16_DIRECT", None)
        else:
            os.environ["KCTC_BF16_DIRECT"] = old
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
