"""The 256-tile streamed direction-split GEMM (gemm_x3p.hip
x3p_bwd_stream256_kernel: the RNN backward's dx and the chained forward's
next-component projection) in isolation, against a numpy float64 product:
C = E[:, :K] Wt0^T + E[:, K:] Wt1^T (+ bias), every producer epoch final.
Both producer orders, with and without the split-K tail slots (whose tiles
sum 1 + 4 partials in a fixed order).  Split-fp16 products: relative error
~1e-6 of the row/column scale."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("forward", [0, 1])
@pytest.mark.parametrize("tail", [0, 1, 3])
@pytest.mark.parametrize("M,N,K", [(256 * 10, 512, 256), (256 * 9 + 16 * 5, 768, 512), (256 * 12, 256, 2048)])
def test_row_stream_matches_float64(kctc, gpu, forward, tail, M, N, K):
    import torch
    rng = np.random.default_rng(M + N + K + 7 * forward + tail)
    E = rng.standard_normal((M, 2 * K)).astype(np.float32)
    Wt = (rng.standard_normal((2, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32) if forward else None
    dE = torch.from_numpy(E).to(gpu)
    dW = torch.from_numpy(Wt).to(gpu)
    dB = torch.from_numpy(bias).to(gpu) if bias is not None else None
    dC = torch.full((M, N), float("nan"), dtype=torch.float32, device=gpu)
    rc = kctc.lib().kcm_test_row_stream(None, M, N, K, forward, tail, dE.data_ptr(), dW.data_ptr(),
                                        dB.data_ptr() if dB is not None else None, dC.data_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    C = dC.cpu().numpy().astype(np.float64)
    ref = E[:, :K].astype(np.float64) @ Wt[0].T.astype(np.float64) + E[:, K:].astype(np.float64) @ Wt[1].T.astype(np.float64)
    if bias is not None:
        ref += bias.astype(np.float64)
    assert np.all(np.isfinite(C))
    scale = np.sqrt(np.mean(ref ** 2))
    err = np.abs(C - ref).max() / scale
    assert err < 2e-5, err
