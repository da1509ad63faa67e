"""kaldi-ctc_amd -- MI355X-native CTC acoustic-model training path.

Host-side mirror of the reference's interfaces over the C-ABI HIP library
libkaldictc_amd.so (built from csrc/ by the Makefile next to this file):

  * warp-ctc ABI (include/ctc.h): compute_ctc_loss / get_workspace_size /
    ctcGetStatusString -- replaces warp-ctc at src/ctc/ctc-nnet-update.cc:211-243.
  * cuDNN-shaped RNN ABI (include/kaldi_rnn.h) -- replaces the
    kaldi::cudnn::Recurrent* shim of src/cudamatrix/cudnn-recurrent.h.
  * nnet2 trainer ABI (include/kaldi_ctc_train.h) -- the NnetCtcUpdater /
    TrainNnetSimple step (src/ctc/ctc-nnet-update.cc:94-128,
    src/ctc/ctc-nnet-train.cc:181-284) on device buffers.
  * egs ABI (include/kaldi_ctc_egs.h) -- NnetCtcExample archives, the
    CompressedMatrix codec, NnetCtcExampleBackgroundReader and FormatNnetInput
    decoded on the GPU (src/ctc/ctc-nnet-example.cc, ctc-nnet-train.cc:31-183,
    ctc-nnet-update.cc:351-424, src/matrix/compressed-matrix.cc).

torch is used only as plumbing (device memory, streams, torch.distributed
rendezvous).  Every entry point fails loudly when the HIP library is missing;
there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkaldictc_amd.so")

CTC_CPU, CTC_GPU = 0, 1
CTC_STATUS = {0: "CTC_STATUS_SUCCESS", 1: "CTC_STATUS_MEMOPS_FAILED", 2: "CTC_STATUS_INVALID_VALUE",
              3: "CTC_STATUS_EXECUTION_FAILED", 4: "CTC_STATUS_UNKNOWN_ERROR"}

_lib = None


class CtcOptions(ctypes.Structure):
    """struct ctcOptions { ctcComputeLocation loc; union { unsigned num_threads;
    hipStream_t stream; }; int blank_label; }  (include/ctc.h)"""
    _fields_ = [("loc", ctypes.c_int), ("stream", ctypes.c_void_p), ("blank_label", ctypes.c_int)]


class CtcError(RuntimeError):
    def __init__(self, status, where):
        msg = lib().ctcGetStatusString(status).decode()
        super().__init__(f"ctcStatus_t {status} : \"{msg}\" returned from '{where}'")
        self.status = status


class KctcError(RuntimeError):
    pass


def build(verbose=False):
    import subprocess
    subprocess.run(["make", "-s" if not verbose else "-j8", "-j8", "-C", HERE], check=True)


def lib():
    """Load libkaldictc_amd.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KctcError(f"{LIB_PATH} is missing: run `make -C {HERE}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, sz = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_size_t
    L.get_warpctc_version.restype = ctypes.c_int
    L.ctcGetStatusString.argtypes = [ctypes.c_int]
    L.ctcGetStatusString.restype = ctypes.c_char_p
    L.compute_ctc_loss.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, CtcOptions]
    L.compute_ctc_loss.restype = ctypes.c_int
    L.get_workspace_size.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, CtcOptions,
                                     ctypes.POINTER(sz)]
    L.get_workspace_size.restype = ctypes.c_int
    L.mictc_compute_ctc_loss_async.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int,
                                               vp, vp, vp, ctypes.c_int]
    L.mictc_compute_ctc_loss_async.restype = ctypes.c_int
    L.mictc_set_frame_group.argtypes = [ctypes.c_int]
    L.mictc_set_frame_group.restype = ctypes.c_int
    if hasattr(L, "mictc_set_win"):  # (absent from pre-round-6 builds run in A/B comparisons)
        L.mictc_set_win.argtypes = [ctypes.c_int]
        L.mictc_set_win.restype = ctypes.c_int
    _bind_optional(L)
    _lib = L
    return L


def _bind_optional(L):
    """Bindings for the RNN / trainer ABIs (added as those layers land)."""
    from . import _bindings  # noqa: F401  (relative import when loaded as a package)
    _bindings.bind(L)


def exported_symbols():
    """Symbols declared by include/*.h (checked by tests/test_abi.py)."""
    import re
    inc = os.path.join(os.path.dirname(HERE), "include")
    names = []
    for fn in sorted(os.listdir(inc)):
        if fn.endswith(".h"):
            txt = open(os.path.join(inc, fn)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            txt = re.sub(r"^\s*typedef[^;]*;", "", txt, flags=re.M)  # function-pointer types are not symbols
            names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-zA-Z_]\w*)\s*\([^;{]*\)\s*;",
                                txt, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "while", "for", "return")))


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


def _stream_handle(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def ctc_frame_group(m=0):
    """Frames per barrier of the alpha/beta kernel (mictc_set_frame_group):
    sets it when m > 0; returns the previous value."""
    return lib().mictc_set_frame_group(int(m))


def ctc_window_kernel(on=-1):
    """Overlapping-window alpha/beta kernel on (1, default) / off (0)
    (mictc_set_win); returns the previous value (on < 0: query only)."""
    return lib().mictc_set_win(int(on))


def ctc_workspace_size(label_lengths, input_lengths, alphabet_size):
    ll = np.ascontiguousarray(label_lengths, dtype=np.int32)
    il = np.ascontiguousarray(input_lengths, dtype=np.int32)
    opts = CtcOptions(CTC_GPU, None, 0)
    out = ctypes.c_size_t()
    st = lib().get_workspace_size(ll.ctypes.data, il.ctypes.data, int(alphabet_size), len(ll),
                                  opts, ctypes.byref(out))
    if st != 0:
        raise CtcError(st, "get_workspace_size")
    return out.value


def compute_ctc_loss(acts, flat_labels, label_lengths, input_lengths, want_grad=True, blank=0,
                     stream=None, workspace=None):
    """warp-ctc compute_ctc_loss on a torch CUDA tensor acts [T, N, A] (float32).
    Returns (costs np.float32 [N], grads tensor or None)."""
    import torch
    assert acts.is_cuda and acts.dtype == torch.float32 and acts.is_contiguous()
    T, N, A = acts.shape
    fl = np.ascontiguousarray(flat_labels, dtype=np.int32)
    if fl.size == 0:
        fl = np.zeros(1, np.int32)
    ll = np.ascontiguousarray(label_lengths, dtype=np.int32)
    il = np.ascontiguousarray(input_lengths, dtype=np.int32)
    if workspace is None:
        workspace = torch.empty(ctc_workspace_size(ll, il, A), dtype=torch.uint8, device=acts.device)
    grads = torch.empty_like(acts) if want_grad else None
    costs = np.zeros(N, np.float32)
    opts = CtcOptions(CTC_GPU, _stream_handle(stream), blank)
    st = lib().compute_ctc_loss(acts.data_ptr(), _ptr(grads), fl.ctypes.data, ll.ctypes.data,
                                il.ctypes.data, A, N, costs.ctypes.data, workspace.data_ptr(), opts)
    if st != 0:
        raise CtcError(st, "compute_ctc_loss")
    return costs, grads


class RnnError(RuntimeError):
    pass


def _krnn_check(st, where):
    if st != 0:
        raise RnnError(f"{where}: {lib().krnnGetStatusString(st).decode()} ({st})")


class Rnn:
    """Thin Python view of the cuDNN-shaped RNN ABI (include/kaldi_rnn.h).

    Mirrors how CuDNNRecurrentComponent drives cudnn-recurrent.h: buffers are
    owned by the caller (torch CUDA tensors here), every call is stream-ordered.
    """
    RELU, TANH, LSTM, GRU = 0, 1, 2, 3

    def __init__(self, mode, input_dim, hidden_dim, num_layers=1, bidirectional=True):
        self.mode, self.D, self.H, self.L = mode, input_dim, hidden_dim, num_layers
        self.dirs = 2 if bidirectional else 1
        h = ctypes.c_void_p()
        _krnn_check(lib().krnnCreate(ctypes.byref(h), mode, input_dim, hidden_dim, num_layers,
                                     1 if bidirectional else 0), "krnnCreate")
        self.h = h

    def set_precision(self, prec):
        """krnnSetPrecision: 0 fp32-class, 1 (or "bf16") bf16 operands."""
        _krnn_check(lib().krnnSetPrecision(self.h, 1 if prec in (1, "bf16") else 0), "krnnSetPrecision")

    def __del__(self):
        try:
            if self.h:
                lib().krnnDestroy(self.h)
        except Exception:
            pass

    @property
    def num_params(self):
        return lib().krnnGetParamsSize(self.h) // 4

    def lin_offset(self, pseudo_layer, lin_id, is_bias):
        dims = (ctypes.c_int * 2)()
        off = lib().krnnGetLinLayerOffset(self.h, pseudo_layer, lin_id, is_bias, dims)
        if off < 0:
            raise RnnError("bad lin layer")
        return off, (dims[0], dims[1])

    def sizes(self, T, N):
        return (lib().krnnGetWorkspaceSize(self.h, T, N), lib().krnnGetTrainingReserveSize(self.h, T, N))

    def forward_training(self, x, w, y, workspace, reserve, stream=None):
        T, N = x.shape[0], x.shape[1]
        _krnn_check(lib().krnnForwardTraining(self.h, _stream_handle(stream), T, N, _ptr(x), _ptr(w),
                                              _ptr(y), _ptr(workspace), workspace.numel(),
                                              _ptr(reserve), reserve.numel()), "krnnForwardTraining")

    def forward_inference(self, x, w, y, workspace, stream=None):
        T, N = x.shape[0], x.shape[1]
        _krnn_check(lib().krnnForwardInference(self.h, _stream_handle(stream), T, N, _ptr(x), _ptr(w),
                                               _ptr(y), _ptr(workspace), workspace.numel()),
                    "krnnForwardInference")

    def backward_data(self, y, dy, w, dx, workspace, reserve, stream=None):
        T, N = y.shape[0], y.shape[1]
        _krnn_check(lib().krnnBackwardData(self.h, _stream_handle(stream), T, N, _ptr(y), _ptr(dy),
                                           _ptr(w), _ptr(dx), _ptr(workspace), workspace.numel(),
                                           _ptr(reserve), reserve.numel()), "krnnBackwardData")

    def backward_weights(self, x, y, dw, workspace, reserve, stream=None):
        T, N = x.shape[0], x.shape[1]
        _krnn_check(lib().krnnBackwardWeights(self.h, _stream_handle(stream), T, N, _ptr(x), _ptr(y),
                                              _ptr(workspace), workspace.numel(), _ptr(dw),
                                              _ptr(reserve), reserve.numel()), "krnnBackwardWeights")

    def device_status(self, stream=None):
        return lib().krnnGetDeviceStatus(self.h, _stream_handle(stream))


def add_mat_mat(C, A, B, transA=False, transB=False, alpha=1.0, beta=0.0, stream=None):
    """C = alpha op(A) op(B) + beta C on 2-D row-major torch CUDA tensors."""
    M, N = C.shape
    K = A.shape[0] if transA else A.shape[1]
    st = lib().kcm_add_mat_mat(_stream_handle(stream), int(transA), int(transB), M, N, K, alpha,
                               _ptr(A), A.stride(0), _ptr(B), B.stride(0), beta, _ptr(C), C.stride(0))
    if st != 0:
        raise KctcError(f"kcm_add_mat_mat failed ({st})")


def add_mat_mat_x3(C, A, B, transA=False, transB=False, alpha=1.0, beta=0.0, stream=None):
    """add_mat_mat on the split-fp16 matrix-core path (kcm_add_mat_mat_x3)."""
    import torch
    M, N = C.shape
    K = A.shape[0] if transA else A.shape[1]
    ws = torch.empty(lib().kcm_add_mat_mat_x3_workspace(M, N, K), dtype=torch.uint8, device=C.device)
    st = lib().kcm_add_mat_mat_x3(_stream_handle(stream), int(transA), int(transB), M, N, K, alpha,
                                  _ptr(A), A.stride(0), _ptr(B), B.stride(0), beta, _ptr(C), C.stride(0),
                                  _ptr(ws))
    if st != 0:
        raise KctcError(f"kcm_add_mat_mat_x3 failed ({st})")


def find_row_max_id(m, stream=None):
    """CuMatrix::FindRowMaxId of a 2-D torch CUDA float32 tensor -> int32
    CUDA tensor (kcm_find_row_max_id: the _find_row_max_id tie rule)."""
    import torch
    assert m.is_cuda and m.dtype == torch.float32 and m.is_contiguous() and m.dim() == 2
    ids = torch.empty(m.shape[0], dtype=torch.int32, device=m.device)
    st = lib().kcm_find_row_max_id(_stream_handle(stream), _ptr(m), m.shape[0], m.shape[1], _ptr(ids))
    if st != 0:
        raise KctcError(f"kcm_find_row_max_id failed ({st})")
    return ids


# ---------------------------------------------------------------------------
# nnet2 trainer (include/kaldi_ctc_train.h)
# ---------------------------------------------------------------------------
def _tcheck(st, where):
    if st != 0:
        raise KctcError(f"{where}: {lib().kctc_last_error().decode()}")


def recipe_config(num_rnn=5, input_dim=40, hidden=512, num_targets=41, rnn_mode=2, bidirectional=True,
                  learning_rate=5e-4, max_seq_length=2000, clipping_threshold=30.0, param_stddev=0.02,
                  bias_stddev=0.2, num_layers=1, norm_based_clipping=True, splice_context=(0,)):
    """Component config lines of the CTC recipe, as written by
    egs/wsj/s5/steps/ctc/nnet2/components.py:73-102 (AddRnnLayer ->
    CuDNNRecurrentComponent + ClipGradientComponent) and an output
    AffineComponent; Splice first (make_configs.py: context 0; any sorted
    offsets containing <= 0 and >= 0 values splice frames)."""
    ctx = [int(c) for c in splice_context]
    lines = [f"SpliceComponent input-dim={input_dim} context={':'.join(map(str, ctx))}"]
    dim = input_dim * len(ctx)
    out = hidden * (2 if bidirectional else 1)
    for _ in range(num_rnn):
        lines.append(f"CuDNNRecurrentComponent input-dim={dim} output-dim={hidden} "
                     f"bidirectional={'true' if bidirectional else 'false'} max-seq-length={max_seq_length} "
                     f"learning-rate={learning_rate} rnn-mode={rnn_mode} num-layers={num_layers} "
                     f"param-stddev={param_stddev} bias-stddev={bias_stddev}")
        lines.append(f"ClipGradientComponent dim={out} clipping-threshold={clipping_threshold} "
                     f"norm-based-clipping={'true' if norm_based_clipping else 'false'}")
        dim = out
    lines.append(f"AffineComponent input-dim={dim} output-dim={num_targets} learning-rate={learning_rate}")
    return "\n".join(lines) + "\n"


class Nnet:
    """nnet2 CTC model on one GPU (the C++ mirror of Nnet + NnetCtcUpdater)."""

    def __init__(self, config=None, seed=0, device=0, _handle=None):
        if _handle is not None:
            self.h = _handle
            return
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_nnet_create(ctypes.byref(h), config.encode(), seed, device), "kctc_nnet_create")
        self.h = h

    @classmethod
    def read(cls, path, device=0):
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_nnet_read(ctypes.byref(h), str(path).encode(), device), "kctc_nnet_read")
        return cls(_handle=h)

    def write(self, path, binary=False):
        """Nnet::Write (nnet-nnet.cc:170-183), Kaldi text or binary mode."""
        _tcheck(lib().kctc_nnet_write_kaldi(self.h, str(path).encode(), int(binary)), "kctc_nnet_write_kaldi")

    @classmethod
    def read_am(cls, path, device=0):
        """nnet2-ctc model file: CtcTransitionModel (kept opaque) + AmNnet (Nnet + priors)."""
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_am_nnet_read(ctypes.byref(h), str(path).encode(), device), "kctc_am_nnet_read")
        return cls(_handle=h)

    def write_am(self, path, binary=True):
        _tcheck(lib().kctc_am_nnet_write(self.h, str(path).encode(), int(binary)), "kctc_am_nnet_write")

    @property
    def priors(self):
        n = lib().kctc_am_nnet_num_priors(self.h)
        out = np.zeros(n, dtype=np.float32)
        _tcheck(lib().kctc_am_nnet_get_priors(self.h, out.ctypes.data, n), "kctc_am_nnet_get_priors")
        return out

    def set_priors(self, priors):
        p = np.ascontiguousarray(priors, dtype=np.float32)
        _tcheck(lib().kctc_am_nnet_set_priors(self.h, p.ctypes.data, p.size), "kctc_am_nnet_set_priors")

    def close(self):
        if getattr(self, "h", None):
            lib().kctc_nnet_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_components(self):
        return lib().kctc_nnet_num_components(self.h)

    def info(self, c):
        buf = ctypes.create_string_buffer(1024)
        _tcheck(lib().kctc_nnet_component_info(self.h, c, buf, 1024), "component_info")
        return buf.value.decode()

    def num_params(self, c):
        return lib().kctc_nnet_num_params(self.h, c)

    def get_params(self, c):
        out = np.zeros(self.num_params(c), np.float32)
        _tcheck(lib().kctc_nnet_get_params(self.h, c, out.ctypes.data, out.size), "get_params")
        return out

    def get_grad(self, c):
        """The gradient component c's last update used (before its clip)."""
        out = np.zeros(self.num_params(c), np.float32)
        _tcheck(lib().kctc_nnet_get_grad(self.h, c, out.ctypes.data, out.size), "get_grad")
        return out

    def set_params(self, c, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        _tcheck(lib().kctc_nnet_set_params(self.h, c, a.ctypes.data, a.size), "set_params")

    def set_learning_rate(self, lr):
        _tcheck(lib().kctc_nnet_set_learning_rate(self.h, lr), "set_learning_rate")

    def clip_stats(self, c):
        a, b = ctypes.c_double(), ctypes.c_double()
        _tcheck(lib().kctc_nnet_clip_stats(self.h, c, ctypes.byref(a), ctypes.byref(b)), "clip_stats")
        return a.value, b.value

    def srand(self, seed):
        """srand(seed) of the trainer's rand() stream (nnet2-ctc-train-simple --srand)."""
        _tcheck(lib().kctc_nnet_srand(self.h, int(seed)), "srand")

    @property
    def rand_calls(self):
        n = ctypes.c_long()
        _tcheck(lib().kctc_nnet_rand_calls(self.h, ctypes.byref(n)), "rand_calls")
        return n.value

    def last_best_path(self, T, N):
        """FindRowMaxId ids [T*N] of the last finished minibatch."""
        out = np.empty(T * N, np.int32)
        _tcheck(lib().kctc_nnet_last_best_path(self.h, out.ctypes.data, out.size), "last_best_path")
        return out

    def last_costs(self, N):
        """Per-utterance CTC costs [N] of the last finished minibatch."""
        out = np.empty(N, np.float64)
        _tcheck(lib().kctc_nnet_last_costs(self.h, out.ctypes.data, N), "last_costs")
        return out

    def last_output(self, T, N, A):
        """Network output [T*N, A] of the last minibatch (host copy)."""
        out = np.empty((T * N, A), np.float32)
        _tcheck(lib().kctc_nnet_last_output(self.h, out.ctypes.data, out.size), "last_output")
        return out

    def _check_feats(self, feats, T, N):
        """feats must hold the FormatNnetInput rows of this network's context:
        T*N*(1 + left + right) rows of input_dim (the C ABI reads exactly that)."""
        l, r = self.context
        rows = T * N * (1 + l + r)
        if feats.dim() != 2 or feats.shape[0] != rows:
            raise KctcError(f"feats has shape {tuple(feats.shape)}; this network (context -{l}..+{r}) reads "
                            f"[T*N*{1 + l + r} = {rows}, input_dim] rows")
        if not feats.is_contiguous():
            raise KctcError("feats must be contiguous")

    def _step(self, fn, feats, T, N, num_frames, flat_labels, label_lengths):
        self._check_feats(feats, T, N)
        nf = np.ascontiguousarray(num_frames, dtype=np.int32)
        fl = np.ascontiguousarray(flat_labels, dtype=np.int32)
        if fl.size == 0:
            fl = np.zeros(1, np.int32)
        ll = np.ascontiguousarray(label_lengths, dtype=np.int32)
        o, a, w = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _tcheck(fn(self.h, _ptr(feats), T, N, nf.ctypes.data, fl.ctypes.data, ll.ctypes.data,
                   ctypes.byref(o), ctypes.byref(a), ctypes.byref(w)), fn.__name__)
        return o.value, a.value, w.value

    @property
    def context(self):
        """(left, right) context of the network (kctc_nnet_context); the input
        of a minibatch has (1 + left + right) rows per output frame."""
        l, r = ctypes.c_int(), ctypes.c_int()
        _tcheck(lib().kctc_nnet_context(self.h, ctypes.byref(l), ctypes.byref(r)), "context")
        return l.value, r.value

    def train_step(self, feats, T, N, num_frames, flat_labels, label_lengths):
        """DoBackprop on one minibatch; feats: device [T*N*num_splice, D] (the
        FormatNnetInput layout, num_splice = 1 + left + right of `context`).
        -> (objf, accuracy, weight)"""
        return self._step(lib().kctc_nnet_train_step, feats, T, N, num_frames, flat_labels, label_lengths)

    def train_step_async(self, feats, T, N, num_frames, flat_labels, label_lengths):
        """Queue a training step (feats must stay alive until its stats come
        back); returns the stats of the minibatch queued before the previous
        one once two are in flight, else None (kctc_nnet_train_step_async).
        feats: device [T*N*num_splice, D] as for train_step."""
        self._check_feats(feats, T, N)
        nf = np.ascontiguousarray(num_frames, dtype=np.int32)
        fl = np.ascontiguousarray(flat_labels, dtype=np.int32)
        if fl.size == 0:
            fl = np.zeros(1, np.int32)
        ll = np.ascontiguousarray(label_lengths, dtype=np.int32)
        h, o, a, w = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _tcheck(lib().kctc_nnet_train_step_async(self.h, _ptr(feats), T, N, nf.ctypes.data, fl.ctypes.data,
                                                 ll.ctypes.data, ctypes.byref(h), ctypes.byref(o),
                                                 ctypes.byref(a), ctypes.byref(w)), "train_step_async")
        return (o.value, a.value, w.value) if h.value else None

    def train_flush(self):
        """Stats of the queued minibatches, oldest first (kctc_nnet_train_flush)."""
        out = []
        while True:
            h, o, a, w = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            _tcheck(lib().kctc_nnet_train_flush(self.h, ctypes.byref(h), ctypes.byref(o), ctypes.byref(a),
                                                ctypes.byref(w)), "train_flush")
            if not h.value:
                return out
            out.append((o.value, a.value, w.value))

    def compute_objf(self, feats, T, N, num_frames, flat_labels, label_lengths):
        """ComputeNnetObjf (no update); feats as for train_step."""
        return self._step(lib().kctc_nnet_compute_objf, feats, T, N, num_frames, flat_labels, label_lengths)

    @property
    def stream(self):
        return lib().kctc_nnet_stream(self.h)

    def set_profiling(self, on):
        _tcheck(lib().kctc_nnet_set_profiling(self.h, int(on)), "set_profiling")

    def profile(self, family):
        ms, n = ctypes.c_double(), ctypes.c_int()
        _tcheck(lib().kctc_nnet_profile(self.h, family.encode(), ctypes.byref(ms), ctypes.byref(n)), "profile")
        return ms.value, n.value

    def propagate(self, feats, T, N, out=None):
        """NnetComputation: network output [T*N, output_dim] (torch CUDA tensor)
        of feats [T*N*num_splice, D] (FormatNnetInput layout)."""
        import torch
        self._check_feats(feats, T, N)
        A = int(self.info(self.num_components - 1).split("output-dim=")[1].split(",")[0])
        if out is None:
            out = torch.empty((T * N, A), dtype=torch.float32, device=feats.device)
        _tcheck(lib().kctc_nnet_propagate(self.h, _ptr(feats), T, N, _ptr(out), out.numel()), "propagate")
        return out

    def decodable(self, feats, T, prob_scale=1.0, blank_threshold=1.0):
        """CtcDecodableAmNnet of one utterance feats [T, D] (plain rows; padded
        for the network's context as pad_input = true) -> np [kept, A]."""
        if feats.dim() != 2 or feats.shape[0] != T or not feats.is_contiguous():
            raise KctcError(f"feats must be a contiguous [T={T}, input_dim] tensor, got {tuple(feats.shape)}")
        A = int(self.info(self.num_components - 1).split("output-dim=")[1].split(",")[0])
        out = np.empty((T, A), np.float32)
        k = ctypes.c_int()
        _tcheck(lib().kctc_am_nnet_decodable(self.h, _ptr(feats), T, prob_scale, blank_threshold, out.ctypes.data,
                                             ctypes.byref(k)), "am_nnet_decodable")
        return out[:k.value].copy()

    def compute_prob(self, rspecifier):
        """nnet2-ctc-compute-prob -> dict(num_examples, tot_like, tot_accuracy, tot_weight)."""
        ne, l, a, w = ctypes.c_long(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _tcheck(lib().kctc_nnet_compute_prob(self.h, str(rspecifier).encode(), ctypes.byref(ne), ctypes.byref(l),
                                             ctypes.byref(a), ctypes.byref(w)), "compute_prob")
        return {"num_examples": ne.value, "tot_like": l.value, "tot_accuracy": a.value, "tot_weight": w.value}

    def set_precision(self, prec):
        """0: fp32-class recurrences / gate GEMMs (default); 1 or "bf16": bf16
        operands, fp32 accumulation (kctc_nnet_set_precision)."""
        prec = 1 if prec in (1, "bf16") else 0
        _tcheck(lib().kctc_nnet_set_precision(self.h, prec), "set_precision")

    def set_momentum(self, m):
        _tcheck(lib().kctc_nnet_set_momentum(self.h, float(m)), "set_momentum")

    def train_simple(self, reader, max_minibatches=0):
        """TrainNnetSimple over an EgsReader -> dict(num_egs, tot_weight, tot_objf, tot_accuracy)."""
        ne, w, o, a = ctypes.c_long(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _tcheck(lib().kctc_nnet_train_simple(self.h, reader._h, int(max_minibatches), ctypes.byref(ne),
                                             ctypes.byref(w), ctypes.byref(o), ctypes.byref(a)), "train_simple")
        return {"num_egs": ne.value, "tot_weight": w.value, "tot_objf": o.value, "tot_accuracy": a.value}

    def enable_dp(self, uid, rank, world):
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        _tcheck(lib().kctc_nnet_enable_dp(self.h, buf, rank, world), "enable_dp")

    def set_dp_mode(self, mode):
        """"grad" (sum the gradients every step) or "average" (independent steps,
        average_params() = nnet-am-average over the ranks)."""
        _tcheck(lib().kctc_nnet_set_dp_mode(self.h, {"grad": 0, "average": 1}[mode]), "set_dp_mode")

    def average_params(self):
        _tcheck(lib().kctc_nnet_average_params(self.h), "average_params")

    def enable_dp_host(self, allreduce, world):
        """Gradient exchange over a host transport: allreduce(np.float32 array)
        must sum it in place across the ranks (e.g. gloo)."""
        def cb(buf, n, user):
            allreduce(np.ctypeslib.as_array(buf, shape=(n,)))
        self._dp_cb = _HOST_ALLREDUCE(cb)  # keep the thunk alive
        _tcheck(lib().kctc_nnet_enable_dp_host(self.h, ctypes.cast(self._dp_cb, ctypes.c_void_p), None, world),
                "enable_dp_host")


    def inject_step_error(self, word=1):
        """Test hook: the next minibatch starts with device error word `word`
        (as after a recurrence timeout): its updates are skipped -- on every
        data-parallel rank -- and the step raises."""
        _tcheck(lib().kctc_nnet_inject_step_error(self.h, int(word)), "inject_step_error")

    def get_component(self, c):
        """A copy of component c (Nnet::GetComponent(c).Copy())."""
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_nnet_get_component(self.h, int(c), ctypes.byref(h)), "kctc_nnet_get_component")
        return Component(_handle=h)

    def set_component(self, c, component):
        """Nnet::SetComponent(c, component.Copy())."""
        _tcheck(lib().kctc_nnet_set_component(self.h, int(c), component.h), "kctc_nnet_set_component")

    def scale_params(self, scale, skip_last_layer=False):
        _tcheck(lib().kctc_nnet_scale_params(self.h, float(scale), int(bool(skip_last_layer))), "scale_params")

    def add_params(self, alpha, other, skip_last_layer=False):
        _tcheck(lib().kctc_nnet_add_params(self.h, float(alpha), other.h, int(bool(skip_last_layer))), "add_params")

    def enable_cu_probe(self, blocks, usec):
        """CU-budget probe: every gradient bucket launches a kernel holding
        `blocks` whole CUs for `usec` us on a comm stream (blocks 0: off)."""
        _tcheck(lib().kctc_nnet_enable_cu_probe(self.h, int(blocks), float(usec)), "enable_cu_probe")


_HOST_ALLREDUCE = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_float), ctypes.c_long, ctypes.c_void_p)


# ---------------------------------------------------------------------------
# nnet2 Component plug-in point (include/kaldi_nnet2_component.h)
# ---------------------------------------------------------------------------
def _torch_sync():
    """The component ABI runs on its own stream: wait for torch's first."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()


class Component:
    """One nnet2 component on the GPU, with the reference's member names
    (src/nnet2/nnet-component.h:157-348): Propagate / Backprop / Copy /
    Write / ReadNew and, for UpdatableComponents, SetZero / DotProduct /
    PerturbParams / Scale / Add / Vectorize / UnVectorize.  Matrices are torch
    CUDA float32 tensors in the time-major [T*N(*num_splice), dim] layout;
    Backprop with a to_update component updates it at once, as the
    reference does (a SetZero(True) copy then holds the gradient)."""

    def __init__(self, config_line=None, seed=0, device=0, _handle=None):
        if _handle is not None:
            self.h = _handle
            return
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_component_init(ctypes.byref(h), config_line.encode(), int(seed), int(device)),
                "kctc_component_init")
        self.h = h

    @classmethod
    def ReadNew(cls, path, device=0):
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_component_read(ctypes.byref(h), str(path).encode(), int(device)), "kctc_component_read")
        return cls(_handle=h)

    def Write(self, path, binary=True):
        _tcheck(lib().kctc_component_write(self.h, str(path).encode(), int(bool(binary))), "kctc_component_write")

    def Copy(self):
        h = ctypes.c_void_p()
        _tcheck(lib().kctc_component_copy(self.h, ctypes.byref(h)), "kctc_component_copy")
        return Component(_handle=h)

    def close(self):
        if getattr(self, "h", None):
            lib().kctc_component_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def Type(self):
        buf = ctypes.create_string_buffer(256)
        _tcheck(lib().kctc_component_type(self.h, buf, 256), "kctc_component_type")
        return buf.value.decode()

    def Info(self):
        buf = ctypes.create_string_buffer(1024)
        _tcheck(lib().kctc_component_info(self.h, buf, 1024), "kctc_component_info")
        return buf.value.decode()

    def _dims(self):
        i, o = ctypes.c_int(), ctypes.c_int()
        _tcheck(lib().kctc_component_dims(self.h, ctypes.byref(i), ctypes.byref(o)), "kctc_component_dims")
        return i.value, o.value

    def InputDim(self):
        return self._dims()[0]

    def OutputDim(self):
        return self._dims()[1]

    def Context(self):
        buf = (ctypes.c_int * 64)()
        n = ctypes.c_int()
        _tcheck(lib().kctc_component_context(self.h, buf, 64, ctypes.byref(n)), "kctc_component_context")
        return list(buf[:n.value])

    def NumSplice(self):
        ctx = self.Context()
        return ctx[-1] - ctx[0] + 1

    def _needs(self):
        i, o = ctypes.c_int(), ctypes.c_int()
        _tcheck(lib().kctc_component_backprop_needs(self.h, ctypes.byref(i), ctypes.byref(o)), "backprop_needs")
        return bool(i.value), bool(o.value)

    def BackpropNeedsInput(self):
        return self._needs()[0]

    def BackpropNeedsOutput(self):
        return self._needs()[1]

    def IsUpdatable(self):
        return bool(lib().kctc_component_is_updatable(self.h))

    def Propagate(self, T, N, inp, out=None):
        """out [T*N, OutputDim] = component(inp [T*N*NumSplice, InputDim])."""
        import torch
        if out is None:
            out = torch.empty((T * N, self.OutputDim()), dtype=torch.float32, device=inp.device)
        _torch_sync()
        _tcheck(lib().kctc_component_propagate(self.h, T, N, _ptr(inp), inp.numel(), _ptr(out), out.numel()),
                "kctc_component_propagate")
        return out

    def Backprop(self, T, N, in_value, out_value, out_deriv, to_update=None, in_deriv=None):
        """Backprop(in_info, out_info, in_value, out_value, out_deriv, to_update,
        in_deriv); in_deriv (a tensor to fill, or None) is returned."""
        _torch_sync()
        _tcheck(lib().kctc_component_backprop(
            self.h, T, N, _ptr(in_value), 0 if in_value is None else in_value.numel(),
            _ptr(out_value), 0 if out_value is None else out_value.numel(), _ptr(out_deriv), out_deriv.numel(),
            None if to_update is None else to_update.h, _ptr(in_deriv),
            0 if in_deriv is None else in_deriv.numel()), "kctc_component_backprop")
        return in_deriv

    # ---- UpdatableComponent ----
    def NumParameters(self):
        return lib().kctc_component_num_params(self.h)

    def Vectorize(self):
        out = np.zeros(self.NumParameters(), np.float32)
        _tcheck(lib().kctc_component_get_params(self.h, out.ctypes.data, out.size), "kctc_component_get_params")
        return out

    def UnVectorize(self, params):
        a = np.ascontiguousarray(params, dtype=np.float32)
        _tcheck(lib().kctc_component_set_params(self.h, a.ctypes.data, a.size), "kctc_component_set_params")

    def LearningRate(self):
        lr = ctypes.c_float()
        _tcheck(lib().kctc_component_learning_rate(self.h, ctypes.byref(lr)), "kctc_component_learning_rate")
        return lr.value

    def SetLearningRate(self, lr):
        _tcheck(lib().kctc_component_set_learning_rate(self.h, float(lr)), "kctc_component_set_learning_rate")

    def IsGradient(self):
        return bool(lib().kctc_component_is_gradient(self.h))

    def SetZero(self, treat_as_gradient):
        _tcheck(lib().kctc_component_set_zero(self.h, int(bool(treat_as_gradient))), "kctc_component_set_zero")

    def DotProduct(self, other):
        d = ctypes.c_double()
        _tcheck(lib().kctc_component_dot_product(self.h, other.h, ctypes.byref(d)), "kctc_component_dot_product")
        return d.value

    def PerturbParams(self, stddev):
        _tcheck(lib().kctc_component_perturb_params(self.h, float(stddev)), "kctc_component_perturb_params")

    def Scale(self, scale):
        _tcheck(lib().kctc_component_scale(self.h, float(scale)), "kctc_component_scale")

    def Add(self, alpha, other):
        _tcheck(lib().kctc_component_add(self.h, float(alpha), other.h), "kctc_component_add")

    def srand(self, seed):
        _tcheck(lib().kctc_component_srand(self.h, int(seed)), "kctc_component_srand")


def set_perturb_seed(seed):
    """Seed of PerturbParams' noise stream (kctc_set_perturb_seed)."""
    _tcheck(lib().kctc_set_perturb_seed(int(seed)), "kctc_set_perturb_seed")


def average_models(nnets, weights=None, skip_last_layer=False):
    """nnet-am-average in process: nnets[0] = sum_i w[i] * nnets[i], with the
    weights normalised to sum to one as GetWeights does (nnet-am-average.cc:
    45-53; default 1/len(nnets)) through the components' Scale / Add."""
    arr = (ctypes.c_void_p * len(nnets))(*[n.h.value if hasattr(n.h, "value") else n.h for n in nnets])
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float32).ravel()
    if w is not None and w.size != len(nnets):
        raise ValueError(f"average_models: {w.size} weights for {len(nnets)} models")
    _tcheck(lib().kctc_nnet_average_models(arr, None if w is None else w.ctypes.data, len(nnets),
                                           int(bool(skip_last_layer))), "kctc_nnet_average_models")


def set_cu_partition(part, nparts):
    """Ranks sharing one device: nnets created afterwards in this process run
    on CU share `part` of `nparts` (kctc_set_cu_partition)."""
    _tcheck(lib().kctc_set_cu_partition(int(part), int(nparts)), "kctc_set_cu_partition")


def cu_partition_probe(part, nparts):
    """The distinct CUs (XCC_ID << 16 | HW_ID[15:8]) a launch on CU share
    `part` of `nparts` runs on (kctc_cu_partition_probe)."""
    ids = np.zeros(4096, dtype=np.uint32)
    n = ctypes.c_int(0)
    _tcheck(lib().kctc_cu_partition_probe(int(part), int(nparts), ids.ctypes.data, ids.size, ctypes.byref(n)),
            "kctc_cu_partition_probe")
    return ids[:n.value].copy()


def softmax_rows(x, stream=None):
    """SoftmaxComponent forward of a 2-D torch CUDA tensor (kctc_softmax_rows)."""
    import torch
    out = torch.empty_like(x)
    _tcheck(lib().kctc_softmax_rows(_stream_handle(stream), _ptr(x), x.shape[0], x.shape[1], _ptr(out)),
            "kctc_softmax_rows")
    return out


def ctc_decodable(probs, priors=None, prob_scale=1.0, blank_threshold=1.0, floor=1e-10, stream=None):
    """CtcDecodableAmNnet's matrix from device probs [T, A] -> torch CUDA [kept, A]."""
    import torch
    T, A = probs.shape
    out = torch.empty_like(probs)
    scratch = torch.empty(lib().kctc_ctc_decodable_scratch_bytes(T), dtype=torch.uint8, device=probs.device)
    k = ctypes.c_int()
    _tcheck(lib().kctc_ctc_decodable(_stream_handle(stream), _ptr(probs), T, A, _ptr(priors), prob_scale,
                                     blank_threshold, floor, _ptr(out), _ptr(scratch), ctypes.byref(k)),
            "kctc_ctc_decodable")
    return out[:k.value]


def dp_unique_id():
    buf = ctypes.create_string_buffer(128)
    _tcheck(lib().kctc_dp_unique_id(buf), "kctc_dp_unique_id")
    return buf.raw


def synth_minibatch(seed, T_max, N, dim, A, label_ratio=0.125, want_feats=True):
    """BASELINE.md §2 synthetic minibatch, already in FormatNnetInput layout."""
    feats = np.empty((T_max * N, dim), np.float32) if want_feats else None
    nf = np.zeros(N, np.int32)
    ll = np.zeros(N, np.int32)
    fl = np.zeros(N * 639 + 1, np.int32)
    n = lib().kctc_synth_minibatch(seed, T_max, N, dim, A, label_ratio,
                                   feats.ctypes.data if feats is not None else None,
                                   nf.ctypes.data, fl.ctypes.data, ll.ctypes.data)
    return feats, nf, fl[:n].copy(), ll


def levenshtein(ref, hyp):
    """kaldi::LevenshteinEditDistance (unit costs) through kctc_levenshtein (host code)."""
    r = np.ascontiguousarray(ref, dtype=np.int32)
    h = np.ascontiguousarray(hyp, dtype=np.int32)
    return lib().kctc_levenshtein(r.ctypes.data, len(r), h.ctypes.data, len(h))


def format_input(utt_feats, T_max=None):
    """FormatNnetInput on a list of [T_n, dim] arrays -> [T_max*N, dim]."""
    N = len(utt_feats)
    dim = utt_feats[0].shape[1]
    nf = np.array([u.shape[0] for u in utt_feats], np.int32)
    T_max = int(T_max or nf.max())
    cat = np.ascontiguousarray(np.concatenate(utt_feats, 0), dtype=np.float32)
    out = np.empty((T_max * N, dim), np.float32)
    _tcheck(lib().kctc_format_input(cat.ctypes.data, nf.ctypes.data, N, dim, T_max, out.ctypes.data),
            "kctc_format_input")
    return out


def smoke_train_step(oracle_lib):
    """One tiny NnetCtcUpdater step (2 x BLSTM-32, N=3, T=24) on cuda:0,
    checked against the fp64 oracle (called from __graft_entry__.smoke())."""
    import torch
    R, H, D, A, T, N, lr = 2, 32, 16, 9, 24, 3, 0.01
    net = Nnet(recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, learning_rate=lr,
                             param_stddev=0.2), seed=11)
    upd = [c for c in range(net.num_components) if net.num_params(c) > 0]
    params = [net.get_params(c).astype(np.float64) for c in upd]
    feats, nf, fl, ll = synth_minibatch(5, T, N, D, A, 0.2)
    objf, acc, wt = net.train_step(torch.from_numpy(feats).to("cuda:0"), T, N, nf, fl, ll)
    s = oracle_lib.NnetSpec()
    s.num_rnn, s.mode, s.hidden, s.dirs, s.layers_per_rnn = R, 2, H, 2, 1
    s.input_dim, s.num_targets = D, A
    s.clip_threshold, s.repair_threshold, s.repair_scale, s.repair_target = 30.0, 0.01, 1.0, 0.0
    s.rnn_clip_gradient, s.lr_rnn, s.lr_affine = 5.0, lr, lr
    Wa, ba = params[-1][:-A].reshape(A, -1).copy(), params[-1][-A:].copy()
    robjf, _, rwt = oracle_lib.train_step(s, params[:-1], Wa, ba, feats.reshape(T, N, D).astype(np.float64),
                                          nf, fl, ll, repair_draws=np.ones(R, np.float32))
    params[-1] = np.concatenate([Wa.ravel(), ba])
    assert abs(objf - robjf) <= 1e-5 * abs(robjf), (objf, robjf)
    for c, p in zip(upd, params):
        got = net.get_params(c).astype(np.float64)
        err = np.linalg.norm(got - p) / np.linalg.norm(p)
        assert err < 1e-5, (c, err)
    net.close()
    return objf, robjf


# ---------------------------------------------------------------------------
# egs: NnetCtcExample archives, CompressedMatrix, background reader, GPU format
# ---------------------------------------------------------------------------
def cm_compress(m):
    """CompressedMatrix::CopyFromMat of a float32 [rows, cols] matrix -> bytes
    (the in-memory image: 20-byte GlobalHeader + body)."""
    m = np.ascontiguousarray(m, dtype=np.float32)
    rows, cols = m.shape
    L = lib()
    out = np.zeros(max(L.kctc_cm_compressed_bytes(rows, cols), 0), dtype=np.uint8)
    if out.size == 0:
        return out
    _tcheck(L.kctc_cm_compress(m.ctypes.data, rows, cols, out.ctypes.data), "kctc_cm_compress")
    return out


def cm_decompress(img):
    """CompressedMatrix::CopyToMat of an image from cm_compress -> float32 [rows, cols]."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    hdr = np.frombuffer(img[:20].tobytes(), dtype=np.int32)
    rows, cols = int(hdr[3]), int(hdr[4])
    out = np.empty((rows, cols), dtype=np.float32)
    _tcheck(lib().kctc_cm_decompress(img.ctypes.data, out.ctypes.data), "kctc_cm_decompress")
    return out


def shuffle_egs(rspecifier, wspecifier, srand=0, buffer_size=0, frame_shift=0, frame_subsampling_factor=0):
    """nnet-ctc-shuffle-egs (src/ctcbin/nnet-ctc-shuffle-egs.cc:25-127) -> examples written."""
    n = ctypes.c_long()
    _tcheck(lib().kctc_egs_shuffle(rspecifier.encode(), wspecifier.encode(), srand, buffer_size, frame_shift,
                                   frame_subsampling_factor, ctypes.byref(n)), "kctc_egs_shuffle")
    return n.value


def sort_egs(rspecifier, wspecifier, srand=0, buffer_size=0):
    """nnet-ctc-sort-egs (src/ctcbin/nnet-ctc-sort-egs.cc:27-133) -> examples written."""
    n = ctypes.c_long()
    _tcheck(lib().kctc_egs_sort(rspecifier.encode(), wspecifier.encode(), srand, buffer_size, ctypes.byref(n)),
            "kctc_egs_sort")
    return n.value


class EgsWriter:
    """NnetCtcExampleWriter over a binary Kaldi archive (features compressed)."""

    def __init__(self, wspecifier):
        self._h = ctypes.c_void_p()
        _tcheck(lib().kctc_egs_writer_open(ctypes.byref(self._h), wspecifier.encode()), "kctc_egs_writer_open")

    def write(self, key, feats, labels, left_context=0, spk_info=None):
        f = np.ascontiguousarray(feats, dtype=np.float32)
        lab = np.ascontiguousarray(labels, dtype=np.int32)
        spk = None if spk_info is None else np.ascontiguousarray(spk_info, dtype=np.float32)
        _tcheck(lib().kctc_egs_write(self._h, key.encode(), f.ctypes.data, f.shape[0], f.shape[1],
                                     lab.ctypes.data, lab.size, left_context,
                                     None if spk is None else spk.ctypes.data, 0 if spk is None else spk.size),
                "kctc_egs_write")

    def close(self):
        if self._h:
            _tcheck(lib().kctc_egs_writer_close(self._h), "kctc_egs_writer_close")
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Minibatch:
    """One minibatch from EgsReader (still compressed until format())."""

    def __init__(self, handle):
        self._h = handle
        L = lib()
        N, T, D, tl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
        _tcheck(L.kctc_minibatch_info(handle, ctypes.byref(N), ctypes.byref(T), ctypes.byref(D), ctypes.byref(tl)),
                "kctc_minibatch_info")
        self.N, self.T_max, self.input_dim, self.total_labels = N.value, T.value, D.value, tl.value
        self.num_splice = L.kctc_minibatch_num_splice(handle)  # rows per output frame of the formatted input
        self.num_frames = np.zeros(self.N, dtype=np.int32)
        self.label_lengths = np.zeros(self.N, dtype=np.int32)
        self.flat_labels = np.zeros(max(self.total_labels, 1), dtype=np.int32)
        _tcheck(L.kctc_minibatch_labels(handle, self.num_frames.ctypes.data, self.label_lengths.ctypes.data,
                                        self.flat_labels.ctypes.data), "kctc_minibatch_labels")
        self.flat_labels = self.flat_labels[:self.total_labels]
        self.keys = [L.kctc_minibatch_key(handle, n).decode() for n in range(self.N)]

    def scratch_bytes(self):
        return int(lib().kctc_minibatch_scratch_bytes(self._h))

    def format(self, out, scratch, stream=None):
        """Stream-ordered FormatNnetInput on the GPU into out [T_max*N*num_splice, input_dim] (device)."""
        _tcheck(lib().kctc_minibatch_format(self._h, _ptr(out), _ptr(scratch), int(scratch.numel()),
                                            ctypes.c_void_p(_stream_handle(stream))), "kctc_minibatch_format")

    def free(self):
        if self._h:
            lib().kctc_minibatch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class EgsReader:
    """SequentialNnetCtcExampleReader + NnetCtcExampleBackgroundReader: iterate
    minibatches (skip rules of ctc-nnet-train.cc:84-95)."""

    def __init__(self, rspecifier, minibatch_size, max_frames=100000, nnet_left_context=0, nnet_right_context=0):
        self._h = ctypes.c_void_p()
        _tcheck(lib().kctc_egs_reader_open(ctypes.byref(self._h), rspecifier.encode(), minibatch_size, max_frames,
                                           nnet_left_context, nnet_right_context), "kctc_egs_reader_open")

    def __iter__(self):
        return self

    def __next__(self):
        mb = ctypes.c_void_p()
        _tcheck(lib().kctc_egs_reader_next(self._h, ctypes.byref(mb)), "kctc_egs_reader_next")
        if not mb.value:
            raise StopIteration
        return Minibatch(mb)

    def stats(self):
        r, k = ctypes.c_long(), ctypes.c_long()
        _tcheck(lib().kctc_egs_reader_stats(self._h, ctypes.byref(r), ctypes.byref(k)), "kctc_egs_reader_stats")
        return r.value, k.value

    def close(self):
        if self._h:
            lib().kctc_egs_reader_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
