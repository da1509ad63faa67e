"""Consumer-gated forward projection (rnn.h rnn_forward_training `side`,
KCTC_FWD_GATE).

The input projection G = x W^T + b of an XCD-pinned split-fp16 forward
recurrence runs on the trainer's side stream CONCURRENTLY with the recurrence
that consumes it: the 256-tile GEMM keeps to the other XCDs, takes its tiles
in the order the two directions need their rows, writes them through and
flags each tile with the call's id; the recurrence's IO waves fetch a row
tile's G rows only once every column tile of it carries that id.  Each tile
is the same GEMM arithmetic as the stream-ordered launch, so training must be
bit-identical to KCTC_FWD_GATE=0: LSTM and GRU, one and two 8-row groups, a
ragged batch (row tiles that straddle steps), and three stacked components
(the first one's projection from the 40-dim input)."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _train(kctc, gpu, cfg, batch, gated, steps=2):
    import torch
    feats, nf, fl, ll, T, N = batch
    old = os.environ.get("KCTC_FWD_GATE")
    os.environ["KCTC_FWD_GATE"] = "1" if gated else "0"
    try:
        net = kctc.Nnet(cfg, seed=5)
        f = torch.from_numpy(feats).to(gpu)
        stats = [net.train_step(f, T, N, nf, fl, ll) for _ in range(steps)]
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.close()
    finally:
        if old is None:
            os.environ.pop("KCTC_FWD_GATE", None)
        else:
            os.environ["KCTC_FWD_GATE"] = old
    return stats, params


@pytest.mark.parametrize("mode,N,T,R", [(2, 16, 400, 3), (3, 16, 300, 2), (2, 13, 350, 2), (2, 8, 301, 2)])
def test_gated_projection_bit_identical(kctc, gpu, mode, N, T, R):
    D, H, A = 40, 512, 41
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                             max_seq_length=T, rnn_mode=mode)
    feats, nf, fl, ll = kctc.synth_minibatch(3 + N, T, N, D, A, 0.125)
    batch = (feats, nf, fl, ll, T, N)
    a = _train(kctc, gpu, cfg, batch, gated=False)
    b = _train(kctc, gpu, cfg, batch, gated=True)
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)
