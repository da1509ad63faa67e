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
    "kcm_add_mat_mat_x3_workspace": (sz, [ci, ci, ci]),
    "kcm_add_mat_mat_x3": (ci, [vp, ci, ci, ci, ci, ci, cf, vp, cl, vp, cl, cf, vp, cl, vp]),
    "kcm_bench_gemm_packed": (cf, [vp, ci, ci, ci, ci, ci, ci]),
    "kcm_find_row_max_id": (ci, [vp, vp, cl, ci, vp]),
    "kcm_clip_gradient_rows": (ci, [vp, vp, cl, ci, cf, vp]),
    "kcm_add_vec_clipped": (ci, [vp, vp, vp, cl, cf, cf]),
    "kcm_add_row_sum_mat": (ci, [vp, vp, cl, ci, cf, cf, vp, vp]),
    # include/kaldi_ctc_train.h
    "kctc_last_error": (ctypes.c_char_p, []),
    "kctc_nnet_create": (ci, [ctypes.POINTER(vp), ctypes.c_char_p, ctypes.c_ulonglong, ci]),
    "kctc_nnet_destroy": (ci, [vp]),
    "kctc_nnet_num_components": (ci, [vp]),
    "kctc_nnet_component_info": (ci, [vp, ci, ctypes.c_char_p, sz]),
    "kctc_nnet_num_params": (cl, [vp, ci]),
    "kctc_nnet_get_params": (ci, [vp, ci, vp, cl]),
    "kctc_nnet_set_params": (ci, [vp, ci, vp, cl]),
    "kctc_nnet_get_grad": (ci, [vp, ci, vp, cl]),
    "kctc_nnet_set_learning_rate": (ci, [vp, cf]),
    "kctc_nnet_clip_stats": (ci, [vp, ci, ctypes.POINTER(cd), ctypes.POINTER(cd)]),
    "kctc_nnet_srand": (ci, [vp, ctypes.c_uint]),
    "kctc_nnet_rand_calls": (ci, [vp, ctypes.POINTER(cl)]),
    "kctc_nnet_last_best_path": (ci, [vp, vp, cl]),
    "kctc_nnet_last_output": (ci, [vp, vp, cl]),
    "kctc_nnet_last_costs": (ci, [vp, vp, ci]),
    "kctc_nnet_train_step": (ci, [vp, vp, ci, ci, vp, vp, vp, ctypes.POINTER(cd), ctypes.POINTER(cd),
                                  ctypes.POINTER(cd)]),
    "kctc_nnet_compute_objf": (ci, [vp, vp, ci, ci, vp, vp, vp, ctypes.POINTER(cd), ctypes.POINTER(cd),
                                    ctypes.POINTER(cd)]),
    "kctc_nnet_train_step_async": (ci, [vp, vp, ci, ci, vp, vp, vp, ip, ctypes.POINTER(cd), ctypes.POINTER(cd),
                                        ctypes.POINTER(cd)]),
    "kctc_nnet_train_flush": (ci, [vp, ip, ctypes.POINTER(cd), ctypes.POINTER(cd), ctypes.POINTER(cd)]),
    "kctc_nnet_stream": (vp, [vp]),
    "kctc_nnet_set_profiling": (ci, [vp, ci]),
    "kctc_nnet_profile": (ci, [vp, ctypes.c_char_p, ctypes.POINTER(cd), ctypes.POINTER(ci)]),
    "kctc_nnet_write": (ci, [vp, ctypes.c_char_p]),
    "kctc_nnet_read": (ci, [ctypes.POINTER(vp), ctypes.c_char_p, ci]),
    "kctc_nnet_write_kaldi": (ci, [vp, ctypes.c_char_p, ci]),
    "kctc_am_nnet_read": (ci, [ctypes.POINTER(vp), ctypes.c_char_p, ci]),
    "kctc_am_nnet_write": (ci, [vp, ctypes.c_char_p, ci]),
    "kctc_am_nnet_num_priors": (ci, [vp]),
    "kctc_am_nnet_get_priors": (ci, [vp, vp, ci]),
    "kctc_am_nnet_set_priors": (ci, [vp, vp, ci]),
    "kctc_dp_unique_id": (ci, [vp]),
    "kctc_nnet_enable_dp": (ci, [vp, vp, ci, ci]),
    "kctc_nnet_enable_dp_host": (ci, [vp, vp, vp, ci]),
    "kctc_nnet_set_dp_mode": (ci, [vp, ci]),
    "kctc_nnet_average_params": (ci, [vp]),
    "kctc_nnet_set_momentum": (ci, [vp, cf]),
    "kctc_nnet_set_precision": (ci, [vp, ci]),
    "krnnSetPrecision": (ci, [vp, ci]),
    "kctc_nnet_train_simple": (ci, [vp, vp, cl, ctypes.POINTER(cl), ctypes.POINTER(cd), ctypes.POINTER(cd),
                                    ctypes.POINTER(cd)]),
    "kctc_levenshtein": (ci, [vp, ci, vp, ci]),
    "kctc_format_input": (ci, [vp, vp, ci, ci, ci, vp]),
    "kctc_synth_minibatch": (cl, [ctypes.c_ulonglong, ci, ci, ci, ci, cd, vp, vp, vp, vp]),
    # include/kaldi_ctc_decode.h
    "kctc_softmax_rows": (ci, [vp, vp, cl, ci, vp]),
    "kctc_ctc_decodable_scratch_bytes": (sz, [ci]),
    "kctc_ctc_decodable": (ci, [vp, vp, ci, ci, vp, cf, cf, cf, vp, vp, ip]),
    "kctc_nnet_propagate": (ci, [vp, vp, ci, ci, vp, cl]),
    "kctc_am_nnet_decodable": (ci, [vp, vp, ci, cf, cf, vp, ip]),
    "kctc_nnet_compute_prob": (ci, [vp, ctypes.c_char_p, ctypes.POINTER(cl), ctypes.POINTER(cd), ctypes.POINTER(cd),
                                    ctypes.POINTER(cd)]),
    # include/kaldi_ctc_egs.h
    "kctc_cm_compressed_bytes": (cl, [ci, ci]),
    "kctc_cm_compress": (ci, [vp, ci, ci, vp]),
    "kctc_cm_decompress": (ci, [vp, vp]),
    "kctc_egs_writer_open": (ci, [ctypes.POINTER(vp), ctypes.c_char_p]),
    "kctc_egs_write": (ci, [vp, ctypes.c_char_p, vp, ci, ci, vp, ci, ci, vp, ci]),
    "kctc_egs_writer_close": (ci, [vp]),
    "kctc_egs_shuffle": (ci, [ctypes.c_char_p, ctypes.c_char_p, ci, ci, ci, ci, ctypes.POINTER(cl)]),
    "kctc_egs_sort": (ci, [ctypes.c_char_p, ctypes.c_char_p, ci, ci, ctypes.POINTER(cl)]),
    "kctc_egs_reader_open": (ci, [ctypes.POINTER(vp), ctypes.c_char_p, ci, ci, ci, ci]),
    "kctc_egs_reader_next": (ci, [vp, ctypes.POINTER(vp)]),
    "kctc_egs_reader_stats": (ci, [vp, ctypes.POINTER(cl), ctypes.POINTER(cl)]),
    "kctc_egs_reader_close": (ci, [vp]),
    "kctc_minibatch_info": (ci, [vp, ip, ip, ip, ctypes.POINTER(cl)]),
    "kctc_minibatch_labels": (ci, [vp, vp, vp, vp]),
    "kctc_minibatch_key": (ctypes.c_char_p, [vp, ci]),
    "kctc_minibatch_scratch_bytes": (cl, [vp]),
    "kctc_minibatch_format": (ci, [vp, vp, vp, cl, vp]),
    "kctc_minibatch_free": (ci, [vp]),
}


def bind(L):
    for name, (res, args) in SIGS.items():
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
