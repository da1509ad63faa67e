"""ctypes view of oracle/liboracle.so -- the CPU checker.

TEST INFRASTRUCTURE: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg only (see oracle/oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None

f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


class NnetSpec(ctypes.Structure):
    _fields_ = [("num_rnn", ctypes.c_int), ("mode", ctypes.c_int), ("hidden", ctypes.c_int),
                ("dirs", ctypes.c_int), ("layers_per_rnn", ctypes.c_int),
                ("input_dim", ctypes.c_int), ("num_targets", ctypes.c_int),
                ("clip_threshold", ctypes.c_float), ("repair_threshold", ctypes.c_float),
                ("repair_scale", ctypes.c_float), ("repair_target", ctypes.c_float),
                ("rnn_clip_gradient", ctypes.c_float), ("lr_rnn", ctypes.c_float),
                ("lr_affine", ctypes.c_float)]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for sfx, rp in (("_f64", f64p), ("_f32", f32p)):
            fn = getattr(L, "oracle_ctc" + sfx)
            fn.argtypes = [rp, ctypes.c_void_p, i32p, i32p, i32p, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, rp, ctypes.c_int]
            fn.restype = None
            fn = getattr(L, "oracle_rnn_forward" + sfx)
            fn.argtypes = [ctypes.c_int] * 7 + [rp, rp, rp, rp]
            fn.restype = None
            fn = getattr(L, "oracle_rnn_backward" + sfx)
            fn.argtypes = [ctypes.c_int] * 7 + [rp, rp, rp, rp, rp, ctypes.c_void_p, ctypes.c_void_p]
            fn.restype = None
            fn = getattr(L, "oracle_train_step" + sfx)
            fn.argtypes = [ctypes.POINTER(NnetSpec), ctypes.c_void_p, rp, rp, rp,
                           ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, ctypes.c_void_p,
                           f64p, f64p, ctypes.POINTER(ctypes.c_double),
                           ctypes.POINTER(ctypes.c_double)]
            fn.restype = ctypes.c_double
            fn = getattr(L, "oracle_train_step_ex" + sfx)
            fn.argtypes = [ctypes.POINTER(NnetSpec), ctypes.c_void_p, rp, rp, rp,
                           ctypes.c_int, ctypes.c_int, i32p, i32p, i32p, ctypes.c_void_p,
                           f64p, f64p, ctypes.POINTER(ctypes.c_double),
                           ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            fn.restype = ctypes.c_double
        for name in ("oracle_rnn_params_size", "oracle_rnn_reserve_size"):
            getattr(L, name).restype = ctypes.c_long
        L.oracle_rnn_params_size.argtypes = [ctypes.c_int] * 5
        L.oracle_rnn_reserve_size.argtypes = [ctypes.c_int] * 6
        L.oracle_rnn_lin_offset.argtypes = [ctypes.c_int] * 8
        L.oracle_rnn_lin_offset.restype = ctypes.c_long
        L.oracle_ctc_accuracy.argtypes = [i32p, ctypes.c_int, ctypes.c_int, i32p, i32p, i32p,
                                          ctypes.POINTER(ctypes.c_double)]
        L.oracle_ctc_accuracy.restype = ctypes.c_double
        L.oracle_levenshtein.argtypes = [i32p, ctypes.c_int, i32p, ctypes.c_int]
        L.oracle_levenshtein.restype = ctypes.c_int
        L.oracle_find_row_max_id_f32.argtypes = [f32p, ctypes.c_int, ctypes.c_int, i32p]
        L.oracle_find_row_max_id_cpu_f32.argtypes = [f32p, ctypes.c_int, ctypes.c_int, i32p]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_softmax_rows_f32.argtypes = [f32p, ctypes.c_long, ctypes.c_int, f32p]
        L.oracle_softmax_rows_f32.restype = None
        L.oracle_ctc_decodable_f32.argtypes = [f32p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_float, f32p]
        L.oracle_ctc_decodable_f32.restype = ctypes.c_int
        _lib = L
    return _lib


def _dt(dtype):
    return ("_f64", np.float64) if np.dtype(dtype) == np.float64 else ("_f32", np.float32)


def ctc(acts, flat_labels, label_lengths, input_lengths, want_grad=True, blank=0):
    """acts [T,N,A] -> (costs [N], grads [T,N,A] or None)."""
    sfx, dt = _dt(acts.dtype)
    acts = np.ascontiguousarray(acts, dtype=dt)
    T, N, A = acts.shape
    costs = np.zeros(N, dtype=dt)
    grads = np.zeros_like(acts) if want_grad else None
    getattr(lib(), "oracle_ctc" + sfx)(
        acts, grads.ctypes.data if grads is not None else None,
        np.ascontiguousarray(flat_labels, dtype=np.int32) if len(flat_labels) else np.zeros(1, np.int32),
        np.ascontiguousarray(label_lengths, dtype=np.int32),
        np.ascontiguousarray(input_lengths, dtype=np.int32), A, N, T, costs, blank)
    return costs, grads


def params_size(mode, D, H, layers, dirs):
    return lib().oracle_rnn_params_size(mode, D, H, layers, dirs)


def lin_offset(mode, D, H, layers, dirs, pl, lin, is_bias):
    return lib().oracle_rnn_lin_offset(mode, D, H, layers, dirs, pl, lin, is_bias)


def rnn_forward(mode, x, w, H, layers, dirs):
    sfx, dt = _dt(x.dtype)
    T, N, D = x.shape
    y = np.zeros((T, N, dirs * H), dtype=dt)
    res = np.zeros(lib().oracle_rnn_reserve_size(mode, T, N, H, layers, dirs), dtype=dt)
    getattr(lib(), "oracle_rnn_forward" + sfx)(mode, T, N, D, H, layers, dirs,
                                              np.ascontiguousarray(x, dtype=dt),
                                              np.ascontiguousarray(w, dtype=dt), y, res)
    return y, res


def rnn_backward(mode, x, w, y, dy, res, H, layers, dirs):
    sfx, dt = _dt(x.dtype)
    T, N, D = x.shape
    dx = np.zeros((T, N, D), dtype=dt)
    dw = np.zeros(w.shape, dtype=dt)
    getattr(lib(), "oracle_rnn_backward" + sfx)(mode, T, N, D, H, layers, dirs,
                                               np.ascontiguousarray(x, dtype=dt),
                                               np.ascontiguousarray(w, dtype=dt), y,
                                               np.ascontiguousarray(dy, dtype=dt), res,
                                               dx.ctypes.data, dw.ctypes.data)
    return dx, dw


def find_row_max_id(m, cpu_rule=False):
    """Best path ids of a [rows, cols] fp32 matrix: the reference CTC path's GPU
    _find_row_max_id tie rule (default) or the CPU FindRowMaxId rule."""
    m = np.ascontiguousarray(m, dtype=np.float32)
    rows, cols = m.shape
    ids = np.empty(rows, np.int32)
    fn = lib().oracle_find_row_max_id_cpu_f32 if cpu_rule else lib().oracle_find_row_max_id_f32
    fn(m, rows, cols, ids)
    return ids


def softmax_rows(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    lib().oracle_softmax_rows_f32(x, x.shape[0], x.shape[1], out)
    return out


def ctc_decodable(probs, priors=None, prob_scale=1.0, blank_threshold=1.0, floor=1e-10):
    """CtcDecodableAmNnet restatement -> [kept, A] log-likelihoods."""
    probs = np.ascontiguousarray(probs, dtype=np.float32)
    T, A = probs.shape
    out = np.empty_like(probs)
    pr = np.ascontiguousarray(priors, dtype=np.float32) if priors is not None else None
    k = lib().oracle_ctc_decodable_f32(probs, T, A, pr.ctypes.data if pr is not None else None, prob_scale,
                                       blank_threshold, floor, out)
    return out[:k].copy()


def accuracy(best_ids, T, N, num_frames, flat_labels, label_lengths):
    w = ctypes.c_double()
    acc = lib().oracle_ctc_accuracy(np.ascontiguousarray(best_ids, dtype=np.int32), T, N,
                                    np.ascontiguousarray(num_frames, dtype=np.int32),
                                    np.ascontiguousarray(flat_labels, dtype=np.int32)
                                    if len(flat_labels) else np.zeros(1, np.int32),
                                    np.ascontiguousarray(label_lengths, dtype=np.int32),
                                    ctypes.byref(w))
    return acc, w.value


def train_step(spec, rnn_params, affine_W, affine_b, feats, num_frames, flat_labels,
               label_lengths, repair_draws=None, clip_num_clipped=None, clip_count=None, extras=None):
    """One NnetCtcUpdater step on the CPU; parameters are updated in place.
    Returns (tot_objf, tot_accuracy, tot_weight).  extras (a dict, optional)
    receives "costs" [N], "logits" [T*N, A] and "ids" [T*N] of the step."""
    sfx, dt = _dt(feats.dtype)
    T, N, D = feats.shape
    C = spec.num_rnn
    arr = (ctypes.c_void_p * C)(*[p.ctypes.data for p in rnn_params])
    cnc = clip_num_clipped if clip_num_clipped is not None else np.zeros(C)
    cc = clip_count if clip_count is not None else np.zeros(C)
    draws = None
    if repair_draws is not None:
        draws = np.ascontiguousarray(repair_draws, dtype=np.float32)
    acc, wt = ctypes.c_double(), ctypes.c_double()
    ex = [None, None, None]
    if extras is not None:
        extras["costs"] = np.zeros(N)
        extras["logits"] = np.zeros((T * N, spec.num_targets), dtype=dt)
        extras["ids"] = np.zeros(T * N, np.int32)
        ex = [extras["costs"].ctypes.data, extras["logits"].ctypes.data, extras["ids"].ctypes.data]
    tot = getattr(lib(), "oracle_train_step_ex" + sfx)(
        ctypes.byref(spec), arr, affine_W, affine_b, np.ascontiguousarray(feats, dtype=dt), T, N,
        np.ascontiguousarray(num_frames, dtype=np.int32),
        np.ascontiguousarray(flat_labels, dtype=np.int32),
        np.ascontiguousarray(label_lengths, dtype=np.int32),
        draws.ctypes.data if draws is not None else None, cnc, cc,
        ctypes.byref(acc), ctypes.byref(wt), *ex)
    return tot, acc.value, wt.value


# ---- CompressedMatrix / FormatNnetInput restatement (oracle/oracle_egs.c) ----
def _egs_bind(L):
    if getattr(L, "_egs_bound", False):
        return
    L.oracle_cm_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    L.oracle_cm_bytes.restype = ctypes.c_long
    L.oracle_cm_compress.argtypes = [f32p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.oracle_cm_compress.restype = ctypes.c_long
    L.oracle_cm_decompress.argtypes = [ctypes.c_void_p, f32p]
    L.oracle_cm_decompress.restype = None
    L.oracle_format_input_cm.argtypes = [ctypes.c_void_p, i32p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, f32p]
    L.oracle_format_input_cm.restype = None
    L._egs_bound = True


def cm_compress(m):
    L = lib()
    _egs_bind(L)
    m = np.ascontiguousarray(m, dtype=np.float32)
    rows, cols = m.shape
    out = np.zeros(max(L.oracle_cm_bytes(rows, cols), 0), dtype=np.uint8)
    if out.size:
        L.oracle_cm_compress(m, rows, cols, out.ctypes.data)
    return out


def cm_decompress(img):
    L = lib()
    _egs_bind(L)
    img = np.ascontiguousarray(img, dtype=np.uint8)
    hdr = np.frombuffer(img[:20].tobytes(), dtype=np.int32)
    out = np.empty((int(hdr[3]), int(hdr[4])), dtype=np.float32)
    L.oracle_cm_decompress(img.ctypes.data, out)
    return out


def format_input_cm(images, ignore, spk, T_max):
    """FormatNnetInput over compressed images -> [T_max*N, dim+spk_dim]."""
    L = lib()
    _egs_bind(L)
    N = len(images)
    imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in images]
    arr = (ctypes.c_void_p * N)(*[i.ctypes.data for i in imgs])
    hdr = np.frombuffer(imgs[0][:20].tobytes(), dtype=np.int32)
    spk = np.ascontiguousarray(spk, dtype=np.float32) if spk is not None else np.zeros((N, 0), np.float32)
    sd = spk.shape[1]
    out = np.empty((T_max * N, int(hdr[4]) + sd), dtype=np.float32)
    L.oracle_format_input_cm(ctypes.cast(arr, ctypes.c_void_p), np.ascontiguousarray(ignore, dtype=np.int32),
                             spk.ctypes.data if sd else None, sd, N, T_max, out)
    return out
