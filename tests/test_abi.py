"""CPU-side checks of the drop-in boundary: the C-ABI library loads without a
GPU and exports every symbol that include/*.h declares; host-only helpers
(FormatNnetInput, the synthetic generator, config lines) behave like the
reference's."""
import ctypes
import subprocess

import numpy as np
import pytest


def test_library_exports_every_declared_symbol(kctc):
    L = kctc.lib()
    declared = kctc.exported_symbols()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    # and they are real dynamic exports of the .so
    out = subprocess.run(["nm", "-D", "--defined-only", kctc.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [s for s in declared if s not in exported]


def test_warpctc_status_strings(kctc):
    L = kctc.lib()
    assert L.ctcGetStatusString(0) == b"no error"
    assert L.ctcGetStatusString(2) == b"invalid value"
    assert L.get_warpctc_version() >= 1


def test_workspace_size_and_invalid_values(kctc):
    L = kctc.lib()
    ll = np.array([3, 0], np.int32)
    il = np.array([10, 7], np.int32)
    sz = kctc.ctc_workspace_size(ll, il, 5)
    assert sz > 4 * 2 * (10 * 7 + 7 * 1)  # at least the alpha/beta spill
    out = ctypes.c_size_t()
    bad = np.array([640, 1], np.int32)  # > MAX_WARPCTC_LABEL_LENGTH
    assert L.get_workspace_size(bad.ctypes.data, il.ctypes.data, 5, 2,
                                kctc.CtcOptions(kctc.CTC_GPU, None, 0), ctypes.byref(out)) == 2
    assert L.get_workspace_size(ll.ctypes.data, il.ctypes.data, 5, 2,
                                kctc.CtcOptions(kctc.CTC_CPU, None, 0), ctypes.byref(out)) == 2


def test_rnn_layout_queries_match_oracle(kctc, oracle):
    for mode in (0, 1, 2, 3):
        for (D, H, L, bi) in ((40, 64, 1, True), (7, 5, 2, True), (12, 8, 2, False)):
            r = kctc.Rnn(mode, D, H, L, bi)
            dirs = 2 if bi else 1
            assert r.num_params == oracle.params_size(mode, D, H, L, dirs)
            nlin = 2 * (4 if mode == 2 else 3 if mode == 3 else 1)
            for pl in range(L * dirs):
                for lin in range(nlin):
                    for isb in (0, 1):
                        off, dims = r.lin_offset(pl, lin, isb)
                        assert off == oracle.lin_offset(mode, D, H, L, dirs, pl, lin, isb)
                        assert dims[0] == H


def test_format_input_time_major(kctc):
    rng = np.random.default_rng(0)
    utts = [rng.standard_normal((t, 3)).astype(np.float32) for t in (5, 2, 4)]
    out = kctc.format_input(utts)
    assert out.shape == (15, 3)
    for n, u in enumerate(utts):
        for t in range(5):
            row = out[t * 3 + n]
            if t < u.shape[0]:
                np.testing.assert_array_equal(row, u[t])
            else:
                assert np.all(row == 0)


def test_synth_minibatch_contract(kctc):
    feats, nf, fl, ll = kctc.synth_minibatch(20161015, 2000, 16, 40, 41, 0.125)
    assert nf[0] == 2000 and np.all(nf >= 1800) and np.all(nf <= 2000)
    assert np.all(ll == np.minimum(np.minimum(np.floor(nf * 0.125), 639), (nf - 1) // 2))
    assert np.all((fl >= 1) & (fl <= 40))
    off = 0
    for L in ll:
        seq = fl[off:off + L]
        assert np.all(seq[1:] != seq[:-1])  # no consecutive repeats (--unique)
        off += L
    f = feats.reshape(2000, 16, 40)
    for n in range(16):
        assert np.all(f[nf[n]:, n] == 0)
    assert abs(f[:nf[0], 0].std() - 1) < 0.05
    again = kctc.synth_minibatch(20161015, 2000, 16, 40, 41, 0.125)
    np.testing.assert_array_equal(again[0], feats)


def _dp_levenshtein(a, b):
    """kaldi::LevenshteinEditDistance restated as the textbook DP (unit costs)."""
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j - 1] + (a[i - 1] != b[j - 1]), prev[j] + 1, cur[j - 1] + 1)
        prev = cur
    return prev[-1]


def test_levenshtein_bitparallel_matches_dp(kctc):
    """ComputeTotAccuracy's edit distance (Myers bit-vector, multi-word refs)
    against the DP, on the shapes the accuracy sees: refs up to 639 labels
    (10 words), hyps with and without the kept leading blank, empty sides."""
    rng = np.random.default_rng(11)
    cases = [([], []), ([], [3, 4]), ([1, 2], []), ([5], [5]), ([5], [6]), ([1, 2, 3], [1, 3]),
             ([0, 1, 2], [1, 2])]
    for m, n, A in ((63, 70, 5), (64, 64, 41), (65, 30, 3), (128, 200, 41), (200, 129, 2), (639, 700, 41)):
        cases.append((list(rng.integers(0, A, m)), list(rng.integers(0, A, n))))
    for m in (1, 17, 64, 100):  # near-identical sequences (small distances)
        a = list(rng.integers(1, 41, m))
        b = list(a)
        for _ in range(3):
            if b:
                b.pop(int(rng.integers(0, len(b))))
            b.insert(int(rng.integers(0, len(b) + 1)), int(rng.integers(0, 41)))
        cases.append((a, b))
    for a, b in cases:
        assert kctc.levenshtein(a, b) == _dp_levenshtein(a, b), (len(a), len(b))


def test_recipe_config_and_bad_configs(kctc):
    cfg = kctc.recipe_config()
    assert cfg.count("CuDNNRecurrentComponent") == 5 and cfg.count("ClipGradientComponent") == 5
    assert "clipping-threshold=30.0 norm-based-clipping=true" in cfg
    # construction needs a device; the config parser errors are checked on the GPU tests
