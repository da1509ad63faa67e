"""Egs preparation tools: nnet-ctc-shuffle-egs and
nnet-ctc-sort-egs through the C ABI (kctc_egs_shuffle / kctc_egs_sort), CPU.

Oracle: a Python restatement of the two tools' loops
(src/ctcbin/nnet-ctc-shuffle-egs.cc:66-115, src/ctcbin/nnet-ctc-sort-egs.cc:66-118)
drawing from glibc's own srand()/rand() through ctypes -- the generator the
reference binaries use via Kaldi's RandInt (base/kaldi-math.cc:100-127) and
libstdc++'s std::random_shuffle (j = rand() % (i + 1)) -- and the frame
subsampling shift (src/ctc/ctc-nnet-example.cc:78-106) on the oracle codec
(oracle/oracle_egs.c).  No reference archive exists in the tree, so the order
is pinned to glibc's generator and the tools' control flow, not to a Kaldi
binary's output ("parity unpinned" against the real tools).  std::sort's order
among equal lengths is implementation-defined; the tests with ties check the
sort property and the multiset only.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

import oracle_lib as O
from test_egs import parse_archive

pytestmark = pytest.mark.timeout(120)

_libc = ctypes.CDLL(ctypes.util.find_library("c"))


def _rand_int(lo, hi):
    """Kaldi RandInt: no draw when hi == lo."""
    if hi == lo:
        return lo
    return lo + _libc.rand() % (hi + 1 - lo)


def oracle_shuffle(keys, seed, buffer_size):
    """Output key order of nnet-ctc-shuffle-egs."""
    _libc.srand(seed)
    if buffer_size == 0:
        egs = list(keys)
        for i in range(1, len(egs)):
            j = _libc.rand() % (i + 1)
            egs[i], egs[j] = egs[j], egs[i]
        return egs
    out, buf = [], [None] * buffer_size
    for k in keys:
        idx = _rand_int(0, buffer_size - 1)
        if buf[idx] is None:
            buf[idx] = k
        else:
            out.append(buf[idx])
            buf[idx] = k
    return out + [k for k in buf if k is not None]


def oracle_sort(keys, frames, buffer_size):
    """Output key order of nnet-ctc-sort-egs (distinct lengths: sort order determined)."""
    by = lambda ks: sorted(ks, key=lambda k: frames[k])
    if buffer_size == 0:
        return by(keys)
    out, buf, num_read = [], [None] * buffer_size, 0
    for k in keys:
        if num_read > 0 and num_read % buffer_size == 0:
            out += by(buf)
            num_read = 0
        buf[num_read] = k
        num_read += 1
    return out + buf[:num_read]  # the last buffer: arrival order, unsorted


def _write_archive(kctc, path, lengths, dim=13, seed=0):
    rng = np.random.default_rng(seed)
    feats = {}
    with kctc.EgsWriter("ark:" + path) as w:
        for i, T in enumerate(lengths):
            key = f"utt{i:04d}"
            f = (rng.standard_normal((T, dim)) * 2 + 0.5).astype(np.float32)
            lab = rng.integers(1, 41, size=max(1, T // 8)).astype(np.int32)
            w.write(key, f, lab, left_context=i % 3, spk_info=None)
            feats[key] = f
    return feats


def _read(path):
    with open(path, "rb") as fh:
        return parse_archive(fh.read())


@pytest.mark.parametrize("seed,buffer_size", [(0, 0), (7, 0), (3, 1), (5, 4), (11, 16), (2, 200)])
def test_shuffle_order_matches_reference_loop(kctc, tmp_path, seed, buffer_size):
    lengths = list(np.random.default_rng(seed).integers(9, 120, size=53))
    _write_archive(kctc, str(tmp_path / "in.ark"), lengths, seed=seed)
    src = {e[0]: e for e in _read(str(tmp_path / "in.ark"))}
    n = kctc.shuffle_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "out.ark"),
                         srand=seed, buffer_size=buffer_size)
    out = _read(str(tmp_path / "out.ark"))
    assert n == len(out) == len(lengths)
    assert [e[0] for e in out] == oracle_shuffle(list(src), seed, buffer_size)
    for key, labels, img, lc, spk in out:  # examples copied unchanged
        s = src[key]
        assert labels.tobytes() == s[1].tobytes() and img.tobytes() == s[2].tobytes() and lc == s[3]


@pytest.mark.parametrize("factor,shift,buffer_size", [(3, 0, 0), (3, 1, 0), (3, 2, 5), (2, 1, 0), (1, 0, 0)])
def test_shuffle_frame_subsampling_shift(kctc, tmp_path, factor, shift, buffer_size):
    lengths = [1, 2, 3, 5, 8, 9, 10, 31, 100, 4]  # format-2 (<= 8 rows) and format-1 images, tiny inputs
    _write_archive(kctc, str(tmp_path / "in.ark"), lengths, seed=factor * 10 + shift)
    src = {e[0]: e for e in _read(str(tmp_path / "in.ark"))}
    kctc.shuffle_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "out.ark"), srand=1,
                     buffer_size=buffer_size, frame_shift=shift, frame_subsampling_factor=factor)
    out = _read(str(tmp_path / "out.ark"))
    assert [e[0] for e in out] == oracle_shuffle(list(src), 1, buffer_size)
    for key, labels, img, lc, spk in out:
        s = src[key]
        assert labels.tobytes() == s[1].tobytes() and lc == s[3]  # supervision untouched
        if factor <= 1:
            assert img.tobytes() == s[2].tobytes()
            continue
        full = O.cm_decompress(s[2])
        rows = [i + shift for i in range(0, full.shape[0], factor) if i + shift < full.shape[0]]
        want = O.cm_compress(full[rows] if rows else full)
        assert img.tobytes() == want.tobytes(), key


def test_shuffle_rejects_bad_shift(kctc, tmp_path):
    _write_archive(kctc, str(tmp_path / "in.ark"), [20, 30])
    with pytest.raises(RuntimeError):
        kctc.shuffle_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "o.ark"), frame_shift=3,
                         frame_subsampling_factor=3)


def test_shuffle_keeps_process_rand_stream(kctc, tmp_path):
    """The library draws from a private glibc state: the host's rand() stream is untouched."""
    _write_archive(kctc, str(tmp_path / "in.ark"), [20, 30, 40, 50])
    _libc.srand(99)
    a = [_libc.rand() for _ in range(3)]
    _libc.srand(99)
    _libc.rand()
    kctc.shuffle_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "o.ark"), srand=5)
    assert [_libc.rand() for _ in range(2)] == a[1:]


@pytest.mark.parametrize("buffer_size", [0, 1, 7, 10, 64])
def test_sort_order_matches_reference_loop(kctc, tmp_path, buffer_size):
    rng = np.random.default_rng(buffer_size)
    lengths = list(rng.permutation(np.arange(10, 10 + 3 * 40, 3))[:40])  # distinct
    _write_archive(kctc, str(tmp_path / "in.ark"), lengths, dim=5)
    src = _read(str(tmp_path / "in.ark"))
    frames = {e[0]: int(np.frombuffer(e[2][12:16].tobytes(), "<i4")[0]) for e in src}
    n = kctc.sort_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "out.ark"),
                      buffer_size=buffer_size)
    out = _read(str(tmp_path / "out.ark"))
    assert n == len(out) == len(src)
    assert [e[0] for e in out] == oracle_sort([e[0] for e in src], frames, buffer_size)
    srcd = {e[0]: e for e in src}
    for key, labels, img, lc, spk in out:
        assert img.tobytes() == srcd[key][2].tobytes() and labels.tobytes() == srcd[key][1].tobytes()


def test_sort_with_ties_is_sorted_permutation(kctc, tmp_path):
    lengths = list(np.random.default_rng(3).integers(10, 16, size=300))  # many ties, > 16 (introsort path)
    _write_archive(kctc, str(tmp_path / "in.ark"), lengths, dim=3)
    kctc.sort_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "out.ark"))
    out = _read(str(tmp_path / "out.ark"))
    got = [int(np.frombuffer(e[2][12:16].tobytes(), "<i4")[0]) for e in out]
    assert got == sorted(lengths)
    assert sorted(e[0] for e in out) == sorted(f"utt{i:04d}" for i in range(300))


def test_tools_on_empty_archive(kctc, tmp_path):
    open(tmp_path / "in.ark", "wb").close()
    assert kctc.shuffle_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "o.ark")) == 0
    assert kctc.sort_egs("ark:" + str(tmp_path / "in.ark"), "ark:" + str(tmp_path / "o2.ark"), buffer_size=3) == 0
