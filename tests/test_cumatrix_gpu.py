"""CuMatrix ops of the path on the GPU vs the oracle, bit for bit where the
result is an index: FindRowMaxId (kcm_find_row_max_id) against the restated
_find_row_max_id (src/cudamatrix/cu-kernels.cu:2454-2500) -- the best path
ComputeTotAccuracy collapses (north_star: bit-exact best-path indices)."""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


def _engineered(rows, cols, seed):
    rng = np.random.default_rng(seed)
    m = rng.integers(-4, 4, size=(rows, cols)).astype(np.float32)  # ties everywhere
    k = rows // 8
    m[:k] = rng.standard_normal((k, cols)).astype(np.float32)      # generic rows
    m[k, :] = -1e20                                                 # nothing above -1e20: -1
    m[k + 1, :] = np.nan                                            # NaN never wins: -1
    m[k + 2, ::3] = -np.inf
    m[k + 3, :] = -3e20
    m[k + 3, cols // 2] = -9.99e19                                  # just above the floor
    m[k + 4, :] = np.inf                                            # all +inf: a tree tie
    if cols > 2:
        m[k + 5, :] = 0.0
        m[k + 5, [1, 2]] = 5.0                                      # tree rule: 2, not 1
    return m


@pytest.mark.parametrize("rows,cols", [(32000, 41), (5000, 1), (3000, 64), (3000, 256), (2000, 300),
                                       (1000, 1000)])
def test_find_row_max_id_bit_exact(kctc, gpu, oracle, rows, cols):
    import torch
    m = _engineered(rows, cols, rows + cols)
    ids = kctc.find_row_max_id(torch.from_numpy(m).to(gpu))
    torch.cuda.synchronize()
    got = ids.cpu().numpy()
    want = oracle.find_row_max_id(m)
    np.testing.assert_array_equal(got, want)
    k = rows // 8
    assert got[k] == -1 and got[k + 1] == -1
    if cols > 2:
        assert got[k + 5] == 2
