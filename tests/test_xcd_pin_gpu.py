"""XCD-pinned recurrences (rnn.hip xcd_mask).

At H = 512 (32 workgroups of 16 units per direction) and N <= 16 every
(row group, direction) of the v6 backward recurrence fits one XCD: the launch
puts it there, exchanges the per-step partial dh through that XCD's L2 (a
ring of two step images), and the streamed dx GEMM keeps off those XCDs and
follows sc1 copies of the recurrence's flags.  Only where the bytes travel
changes, not the arithmetic: the trained parameters must equal the
unpinned run's (KCTC_XCD6=0) bit for bit, for LSTM and GRU, BLSTM with one
and two row groups, a ragged minibatch, and the configs[2] shape (N = 64:
four row groups x two directions of 16 workgroups, one per XCD).  The forward recurrence pins the
same way (KCTC_XCD6F): its h hand-off through a ring of two L2-resident step
images, the per-step images written through for the next component's
streamed projection, which follows sc1 copies of the epochs."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _train(kctc, gpu, cfg, batch, pinned, steps=2, var="KCTC_XCD6"):
    import torch
    feats, nf, fl, ll, T, N = batch
    old = os.environ.get(var)
    os.environ[var] = "1" if pinned else "0"
    try:
        net = kctc.Nnet(cfg, seed=11)
        f = torch.from_numpy(feats).to(gpu)
        stats = [net.train_step(f, T, N, nf, fl, ll) for _ in range(steps)]
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
        net.close()
    finally:
        if old is None:
            os.environ.pop(var, None)
        else:
            os.environ[var] = old
    return stats, params


@pytest.mark.parametrize("var", ["KCTC_XCD6", "KCTC_XCD6F", "KCTC_XCD6F-stk"])
@pytest.mark.parametrize("mode,N,T", [(2, 16, 400), (2, 8, 300), (3, 16, 300), (2, 13, 350),
                                      # configs[2]: four 16-row groups of U = 32 (16 workgroups a
                                      # direction): eight slots of 16 workgroups, one per XCD
                                      (2, 64, 200), (3, 64, 160), (2, 57, 180)])
def test_pinned_bit_identical(kctc, gpu, mode, N, T, var):
    D, H, A, R = 40, 512, 41, 2
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                             max_seq_length=T, rnn_mode=mode)
    feats, nf, fl, ll = kctc.synth_minibatch(7 + N, T, N, D, A, 0.125)
    batch = (feats, nf, fl, ll, T, N)
    # KCTC_XCD6F: the IO-wave forward, whose pinned form feeds a streamed
    # projection here (KCTC_FWD_STREAM_PINNED, off by default: rnn.hip
    # chain_ok) as its unpinned form does; KCTC_XCD6F-stk: the default
    # stacked forward of <= 8-row groups, projections after the recurrence
    env = {"KCTC_FWD_STREAM_PINNED": "1"}
    if var == "KCTC_XCD6F":
        env["KCTC_STK_FWD"] = "0"
    elif var == "KCTC_XCD6F-stk":
        env = {"KCTC_FWD_STREAM": "0"}
        var = "KCTC_XCD6F"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        a = _train(kctc, gpu, cfg, batch, pinned=False, var=var)
        b = _train(kctc, gpu, cfg, batch, pinned=True, var=var)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("mode", [2, 3])
def test_stacked_hilo_matches_oracle_grade(kctc, gpu, mode):
    """KCTC_STK=1 (rnn.hip kPrecX3S: hi / lo of a <= 8-row group stacked in one
    MFMA operand, all four split products) against the default 3-MFMA form:
    not bit-identical (different products and order), but the two agree to
    fp32-class accuracy after two training steps."""
    D, H, A, R, N, T = 40, 512, 41, 2, 16, 300
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=5e-4,
                             max_seq_length=T, rnn_mode=mode)
    feats, nf, fl, ll = kctc.synth_minibatch(5, T, N, D, A, 0.125)
    batch = (feats, nf, fl, ll, T, N)
    a = _train(kctc, gpu, cfg, batch, pinned=False, var="KCTC_STK")
    b = _train(kctc, gpu, cfg, batch, pinned=True, var="KCTC_STK")
    for x, y in zip(a[1], b[1]):
        err = np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-30)
        assert err < 1e-5, err
