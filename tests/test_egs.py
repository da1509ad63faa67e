"""egs path: CompressedMatrix codec, NnetCtcExample archives, the background
minibatch reader (CPU) and FormatNnetInput decoded on the GPU (gpu).

Oracle: oracle/oracle_egs.c (CPU restatement of src/matrix/compressed-matrix.cc
and of FormatNnetInput, src/ctc/ctc-nnet-update.cc:351-424).  No reference
archive or codec output exists in the reference tree, so the codec parity is
"unpinned" against a Kaldi binary; it is pinned by the reference's own
property tests (src/matrix/matrix-lib-test.cc:4126-4297, mirrored below) and
the archive layout by an independent Python writer/parser of the Kaldi binary
token stream (base/io-funcs-inl.h, ctc-nnet-example.cc:29-60).
"""
import struct

import numpy as np
import pytest

import oracle_lib as O


# ---------------------------------------------------------------------------
# independent Kaldi binary archive writer / parser (test side)
# ---------------------------------------------------------------------------
def _int(v):
    return bytes([4]) + struct.pack("<i", v)


def eg_bytes(key, labels, left_context=0, spk=None, cm=None, plain=None):
    b = key.encode() + b" \0B<NnetCtcExample> <Labels> "
    lab = np.asarray(labels, dtype="<i4")
    b += bytes([4]) + struct.pack("<i", lab.size) + lab.tobytes()
    b += b"<InputFrames> "
    if plain is not None:
        m = np.ascontiguousarray(plain, dtype="<f4")
        b += b"FM " + _int(m.shape[0]) + _int(m.shape[1]) + m.tobytes()
    else:
        fmt = struct.unpack("<i", cm[:4].tobytes())[0]
        b += (b"CM " if fmt == 1 else b"CM2 ") + cm[4:].tobytes()
    b += b"<LeftContext> " + _int(left_context)
    spk = np.zeros(0, dtype="<f4") if spk is None else np.asarray(spk, dtype="<f4")
    b += b"<SpkInfo> FV " + _int(spk.size) + spk.tobytes()
    b += b"</NnetCtcExample> "
    return b


def parse_archive(data):
    out, i = [], 0

    def tok():
        nonlocal i
        j = data.index(b" ", i)
        t = data[i:j].decode()
        i = j + 1
        return t

    def integer():
        nonlocal i
        assert data[i] == 4
        v = struct.unpack("<i", data[i + 1:i + 5])[0]
        i += 5
        return v

    while i < len(data):
        key = tok()
        assert data[i:i + 2] == b"\0B"
        i += 2
        assert tok() == "<NnetCtcExample>" and tok() == "<Labels>"
        n = integer()
        labels = np.frombuffer(data[i:i + 4 * n], dtype="<i4").copy()
        i += 4 * n
        assert tok() == "<InputFrames>"
        t = tok()
        rows, cols = struct.unpack("<ii", data[i + 8:i + 16])
        fmt = 1 if t == "CM" else 2
        body = cols * (8 + rows) if fmt == 1 else 2 * rows * cols
        img = np.frombuffer(struct.pack("<i", fmt) + data[i:i + 16 + body], dtype=np.uint8).copy()
        i += 16 + body
        assert tok() == "<LeftContext>"
        lc = integer()
        assert tok() == "<SpkInfo>" and tok() == "FV"
        n = integer()
        spk = np.frombuffer(data[i:i + 4 * n], dtype="<f4").copy()
        i += 4 * n
        assert tok() == "</NnetCtcExample>"
        out.append((key, labels, img, lc, spk))
    return out


def pathological(rng, n):
    """UnitTestCompressedMatrix's generator (matrix-lib-test.cc:4136-4162)."""
    rows, cols = int(rng.integers(0, 20)), int(rng.integers(0, 15))
    if rows * cols == 0:
        return None
    if rng.integers(0, 2) == 0:
        cols = 1 + int(rng.integers(0, 3))
    if rng.integers(0, 3) != 0:
        m = rng.standard_normal((rows, cols))
    else:
        m = np.full((rows, cols), rng.standard_normal())
    if rng.integers(0, 2) == 0:
        m[rng.integers(0, rows)] = rng.standard_normal() * 4.0
    val = rng.standard_normal() * 4.0
    mod = 1 + int(rng.integers(0, 5))
    mask = rng.integers(0, mod, size=(rows, cols)) != 0
    m[mask] = val
    return m.astype(np.float32)


# ---------------------------------------------------------------------------
# codec
# ---------------------------------------------------------------------------
def test_codec_bit_exact_vs_oracle(kctc):
    rng = np.random.default_rng(1)
    shapes = [(100, 40), (2000, 40), (9, 5), (8, 40), (1, 1), (4, 3), (5, 2), (1, 40), (301, 13)]
    mats = [rng.standard_normal(s).astype(np.float32) * 3 + 1 for s in shapes]
    mats += [np.full((20, 4), 2.5, np.float32), np.zeros((12, 3), np.float32), np.full((3, 3), -7.0, np.float32)]
    for n in range(600):
        m = pathological(rng, n)
        if m is not None:
            mats.append(m)
    for m in mats:
        a, b = kctc.cm_compress(m), O.cm_compress(m)
        assert a.tobytes() == b.tobytes(), m.shape
        np.testing.assert_array_equal(kctc.cm_decompress(a), O.cm_decompress(b))


def test_codec_reference_properties(kctc):
    """matrix-lib-test.cc:4126-4297: ||M2 - M|| <= 0.015 ||M|| and re-compressing
    M2 reproduces M2 to 1e-4, each with at most a couple of failures."""
    rng = np.random.default_rng(2)
    fail_err = fail_idem = tot = 0
    for n in range(2000):
        m = pathological(rng, n)
        if m is None:
            continue
        tot += 1
        m2 = kctc.cm_decompress(kctc.cm_compress(m))
        assert m2.shape == m.shape
        if np.linalg.norm(m2 - m) > 0.015 * np.linalg.norm(m):
            fail_err += 1
        m3 = kctc.cm_decompress(kctc.cm_compress(m2))
        if not np.abs(m3 - m2).max() <= 1e-4 * max(1.0, np.abs(m2).max()):
            fail_idem += 1
    assert tot > 1000
    assert fail_err <= 2 and fail_idem <= 2, (fail_err, fail_idem)


def test_codec_rejects_nonfinite(kctc):
    m = np.ones((10, 3), np.float32)
    m[2, 1] = np.inf
    with pytest.raises(kctc.KctcError):
        kctc.cm_compress(m)


# ---------------------------------------------------------------------------
# archives + background reader
# ---------------------------------------------------------------------------
def _make_egs(rng, n, dim=40, T=(30, 200), spk_dim=0, left_context=0):
    egs = []
    for i in range(n):
        t = int(rng.integers(*T))
        L = min(int(rng.integers(0, max(1, (t - 1) // 2))), 639)  # readable: <= 639 labels
        feats = rng.standard_normal((t, dim)).astype(np.float32)
        labels = rng.integers(1, 41, size=L).astype(np.int32)
        spk = rng.standard_normal(spk_dim).astype(np.float32) if spk_dim else None
        egs.append((f"utt{i:04d}", feats, labels, left_context, spk))
    return egs


def test_writer_layout_matches_independent_parser(kctc, tmp_path):
    rng = np.random.default_rng(3)
    egs = _make_egs(rng, 7, spk_dim=3, left_context=2)
    egs.append(("short-utt", rng.standard_normal((6, 40)).astype(np.float32), np.array([3], np.int32), 0,
                rng.standard_normal(3).astype(np.float32)))  # <= 8 rows: CM2
    path = str(tmp_path / "egs.ark")
    with kctc.EgsWriter("ark:" + path) as w:
        for key, f, lab, lc, spk in egs:
            w.write(key, f, lab, lc, spk)
    parsed = parse_archive(open(path, "rb").read())
    assert len(parsed) == len(egs)
    for (key, f, lab, lc, spk), (k2, l2, img, lc2, s2) in zip(egs, parsed):
        assert key == k2 and lc == lc2
        np.testing.assert_array_equal(lab, l2)
        np.testing.assert_array_equal(spk, s2)
        assert img.tobytes() == O.cm_compress(f).tobytes()


def test_reader_parses_independent_archive(kctc, tmp_path):
    rng = np.random.default_rng(4)
    egs = _make_egs(rng, 10)
    data = b""
    for i, (key, f, lab, lc, spk) in enumerate(egs):
        if i == 3:
            data += eg_bytes(key, lab, lc, spk, plain=f)  # uncompressed "FM": compressed on read
        else:
            data += eg_bytes(key, lab, lc, spk, cm=O.cm_compress(f))
    path = tmp_path / "in.ark"
    path.write_bytes(data)
    r = kctc.EgsReader(str(path), minibatch_size=4, max_frames=100000)
    mbs = list(r)
    assert [m.N for m in mbs] == [4, 4, 2]
    keys = [k for m in mbs for k in m.keys]
    assert keys == [e[0] for e in egs]
    i = 0
    for m in mbs:
        off = 0
        for n in range(m.N):
            key, f, lab, lc, spk = egs[i]
            assert m.num_frames[n] == f.shape[0]
            assert m.label_lengths[n] == lab.size
            np.testing.assert_array_equal(m.flat_labels[off:off + lab.size], lab)
            off += lab.size
            i += 1
        assert m.T_max == max(m.num_frames) and m.input_dim == 40
    assert r.stats() == (10, 0)
    r.close()


def test_reader_skip_rules(kctc, tmp_path):
    """ctc-nnet-train.cc:84-95: skip num_frames > max_frames, labels > 639,
    num_frames < 2*labels + 1."""
    rng = np.random.default_rng(5)
    f = lambda t: rng.standard_normal((t, 40)).astype(np.float32)  # noqa: E731
    cases = [("ok1", f(100), np.arange(1, 11)),
             ("too-long", f(400), np.arange(1, 11)),          # > max_frames = 300
             ("tight", f(21), np.arange(1, 11)),              # 21 = 2*10+1: kept
             ("too-few-frames", f(20), np.arange(1, 11)),     # 20 < 21: skipped
             ("too-many-labels", f(290), np.ones(640)),       # > 639 (also fails 2L+1)
             ("ok2", f(50), np.zeros(0))]
    path = str(tmp_path / "s.ark")
    with kctc.EgsWriter(path) as w:
        for key, feats, lab in cases:
            w.write(key, feats, np.asarray(lab, np.int32))
    r = kctc.EgsReader(path, minibatch_size=16, max_frames=300)
    mbs = list(r)
    assert len(mbs) == 1 and mbs[0].keys == ["ok1", "tight", "ok2"]
    assert r.stats() == (3, 3)


def test_reader_errors(kctc, tmp_path):
    with pytest.raises(kctc.KctcError):
        kctc.EgsReader(str(tmp_path / "missing.ark"), 4)
    bad = tmp_path / "text.ark"
    bad.write_bytes(b"utt1 <NnetCtcExample> <Labels> [ 1 2 ]\n")
    r = kctc.EgsReader(str(bad), 4)
    with pytest.raises(kctc.KctcError):
        next(iter(r))
    empty = tmp_path / "empty.ark"
    empty.write_bytes(b"")
    assert list(kctc.EgsReader(str(empty), 4)) == []


# ---------------------------------------------------------------------------
# GPU: FormatNnetInput decode + pack
# ---------------------------------------------------------------------------
def _gpu_format(kctc, mb, dev):
    import torch
    out = torch.full((mb.T_max * mb.N, mb.input_dim), float("nan"), dtype=torch.float32, device=dev)
    scratch = torch.empty(mb.scratch_bytes(), dtype=torch.uint8, device=dev)
    mb.format(out, scratch)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("spk_dim,left_context,N,T", [(0, 0, 16, (1700, 2001)), (5, 3, 7, (4, 60)),
                                                      (0, 0, 64, (300, 700)), (2, 0, 3, (2, 12))])
def test_gpu_format_bit_exact(kctc, gpu, tmp_path, spk_dim, left_context, N, T):
    rng = np.random.default_rng(6 + N)
    egs = _make_egs(rng, N, spk_dim=spk_dim, left_context=left_context, T=T)
    path = str(tmp_path / "g.ark")
    with kctc.EgsWriter(path) as w:
        for key, f, lab, lc, spk in egs:
            w.write(key, f, lab, lc, spk)
    mb = next(iter(kctc.EgsReader(path, minibatch_size=N, max_frames=100000)))
    got = _gpu_format(kctc, mb, gpu)
    imgs = [O.cm_compress(e[1]) for e in egs]
    spk = np.stack([e[4] for e in egs]) if spk_dim else None
    ref = O.format_input_cm(imgs, [left_context] * N, spk, mb.T_max)
    assert mb.T_max == max(e[1].shape[0] for e in egs) - left_context
    np.testing.assert_array_equal(got, ref)


@pytest.mark.gpu
def test_train_from_egs_matches_host_formatted(kctc, gpu, tmp_path):
    """A train step on GPU-formatted egs equals one on the oracle-formatted
    features (identical bytes in -> identical objf out)."""
    import torch
    rng = np.random.default_rng(9)
    N, D = 4, 40
    egs = _make_egs(rng, N, dim=D, T=(60, 120))
    path = str(tmp_path / "t.ark")
    with kctc.EgsWriter(path) as w:
        for key, f, lab, lc, spk in egs:
            w.write(key, f, lab, lc, spk)
    mb = next(iter(kctc.EgsReader(path, minibatch_size=N)))
    cfg = kctc.recipe_config(num_rnn=2, input_dim=D, hidden=32, num_targets=41, max_seq_length=200)
    a = kctc.Nnet(cfg, seed=7, device=0)
    b = kctc.Nnet(cfg, seed=7, device=0)
    feats = torch.empty((mb.T_max * N, D), dtype=torch.float32, device=gpu)
    scratch = torch.empty(mb.scratch_bytes(), dtype=torch.uint8, device=gpu)
    mb.format(feats, scratch, stream=a.stream)
    ra = a.train_step(feats, mb.T_max, N, mb.num_frames, mb.flat_labels, mb.label_lengths)
    ref = O.format_input_cm([O.cm_compress(e[1]) for e in egs], [0] * N, None, mb.T_max)
    fb = torch.from_numpy(ref).to(gpu)
    torch.cuda.synchronize()
    rb = b.train_step(fb, mb.T_max, N, mb.num_frames, mb.flat_labels, mb.label_lengths)
    assert ra == rb
