"""ctypes signatures for the RNN, CuMatrix and trainer ABIs (include/kaldi_rnn.h,
include/kaldi_cumatrix.h, include/kaldi_ctc_train.h).  Bound only when the
symbol exists so that a partially built library still loads; callers fail
loudly on a missing one."""
import ctypes

vp, ci, cl, cf, cd, sz = (ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float,
                          ctypes.c_double, ctypes.c_size_t)
ip = ctypes.POINTER(ctypes.c_int)

SIGS = {
    # include/kaldi_rnn.h
    "krnnCreate": (ci, [ctypes.POINTER(vp), ci, ci, ci, ci, ci]),
    "krnnDestroy": (ci, [vp]),
    "krnnGetStatusString": (ctypes.c_char_p, [ci]),
    "krnnGetParamsSize": (sz, [vp]),
    "krnnGetLinLayerOffset": (cl, [vp, ci, ci, ci, ip]),
    "krnnGetWorkspaceSize": (sz, [vp, ci, ci]),
    "krnnGetTrainingReserveSize": (sz, [vp, ci, ci]),
    "krnnForwardTraining": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, sz, vp, sz]),
    "krnnForwardInference": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, sz]),
    "krnnBackwardData": (ci, [vp, vp, ci, ci, vp, vp, vp, vp, vp, sz, vp, sz]),
    "krnnBackwardWeights": (ci, [vp, vp, ci, ci, vp, vp, vp, sz, vp, vp, sz]),
    "krnnGetDeviceStatus": (ci, [vp, vp]),
    # include/kaldi_cumatrix.h
    "kcm_add_mat_mat": (ci, [vp, ci, ci, ci, ci, ci, cf, vp, cl, vp, cl, cf, vp, cl]),
    "kcm_find_row_max_id": (ci, [vp, vp, cl, ci, vp]),
    "kcm_clip_gradient_rows": (ci, [vp, vp, cl, ci, cf, vp]),
    "kcm_add_vec_clipped": (ci, [vp, vp, vp, cl, cf, cf]),
    "kcm_add_row_sum_mat": (ci, [vp, vp, cl, ci, cf, cf, vp, vp]),
}


def bind(L):
    for name, (res, args) in SIGS.items():
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
