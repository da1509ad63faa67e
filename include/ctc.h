/*
 * ctc.h -- warp-ctc compatible C ABI, implemented by libkaldictc_amd.so with
 * hand-written CDNA4 (gfx950) HIP kernels.
 *
 * Replaces the external warp-ctc library that the reference includes as
 *     extern "C" { #include "ctc.h" }          src/ctc/ctc-nnet-update.cc:27-29
 * and calls as
 *     get_workspace_size(...)                  src/ctc/ctc-nnet-update.cc:211-214
 *     compute_ctc_loss(...)  (grads / NULL)    src/ctc/ctc-nnet-update.cc:224-243
 *     ctcGetStatusString(ret)                  src/ctc/ctc-nnet-update.cc:31-37
 * The declarations reproduce the public upstream warp-ctc API (baidu-research
 * warp-ctc include/ctc.h, which the lifeiteng fork installed by
 * tools/extras/install_warp_ctc.sh:8-11 keeps); CUstream becomes hipStream_t.
 *
 * Contract (unchanged from warp-ctc):
 *  - activations [maxT][minibatch][alphabet_size] float, DEVICE, C-order,
 *    maxT = max(input_lengths); un-normalised (softmax is applied inside).
 *  - gradients   same shape, DEVICE, nullable; d(-log p)/d activations.  Rows
 *    t >= input_lengths[n] are written with 0 (the caller need not pre-zero).
 *  - flat_labels, label_lengths, input_lengths, costs: HOST pointers.
 *    costs[n] = -log p(labels_n | x_n), filled when the call returns (the call
 *    synchronises options.stream).  An utterance with L + repeats > T gets
 *    cost 0 and a zero gradient (warp-ctc's CPU behaviour).
 *  - workspace: DEVICE, >= get_workspace_size() bytes, owned by the caller.
 *  - loc must be CTC_GPU: this build has no CPU compute path (a CTC_CPU call
 *    returns CTC_STATUS_INVALID_VALUE).
 */
#ifndef KALDI_CTC_AMD_CTC_H_
#define KALDI_CTC_AMD_CTC_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;
typedef struct ihipStream_t *ctcStream_t; /* == hipStream_t */

typedef enum {
  CTC_STATUS_SUCCESS = 0,
  CTC_STATUS_MEMOPS_FAILED = 1,
  CTC_STATUS_INVALID_VALUE = 2,
  CTC_STATUS_EXECUTION_FAILED = 3,
  CTC_STATUS_UNKNOWN_ERROR = 4
} ctcStatus_t;

typedef enum { CTC_CPU = 0, CTC_GPU = 1 } ctcComputeLocation;

struct ctcOptions {
  ctcComputeLocation loc;
  union {
    unsigned int num_threads; /* CTC_CPU (unsupported here) */
    ctcStream_t stream;       /* CTC_GPU */
  };
  int blank_label;
};

int get_warpctc_version(void);
const char *ctcGetStatusString(ctcStatus_t status);

ctcStatus_t compute_ctc_loss(const float *const activations, float *gradients,
                             const int *const flat_labels, const int *const label_lengths,
                             const int *const input_lengths, int alphabet_size,
                             int minibatch, float *costs, void *workspace,
                             struct ctcOptions options);

ctcStatus_t get_workspace_size(const int *const label_lengths,
                               const int *const input_lengths, int alphabet_size,
                               int minibatch, struct ctcOptions info,
                               size_t *size_bytes);

/* ---- extensions (not in upstream warp-ctc) ------------------------------
 * Stream-ordered variant used by the native trainer: identical math, but
 * costs_dev (double[minibatch], DEVICE) is written asynchronously and the
 * call never synchronises, so a whole train step can be captured/queued
 * without host round trips.  Host arrays are consumed before return. */
ctcStatus_t mictc_compute_ctc_loss_async(const float *activations, float *gradients,
                                         const int *flat_labels, const int *label_lengths,
                                         const int *input_lengths, int alphabet_size,
                                         int minibatch, double *costs_dev, void *workspace,
                                         ctcStream_t stream, int blank_label);

/* TEST / TUNING KNOB, not part of the warp-ctc contract: frames per barrier
 * of the alpha/beta recursion (1..8; default 8, or KCTC_CTC_PAIR read once at
 * the first call).  PROCESS-GLOBAL: every later launch from any thread or
 * network reads it, so set it only while no CTC call is in flight (the tests
 * do, one process).  Returns the previous value; m <= 0 only queries.  Same
 * results for every m (tests/test_ctc_gpu.py). */
int mictc_set_frame_group(int m);

/* TEST KNOB, not part of the warp-ctc contract: 1 (default) runs the
 * alpha/beta recursion on overlapping per-wave state windows (one
 * log-sum-exp per lane and frame, up to 12 waves), 0 on the 512-thread kernel
 * with halo log-sum-exps.  Process-global like mictc_set_frame_group; same
 * results either way (tests/test_ctc_gpu.py).  Returns the previous value;
 * on < 0 only queries. */
int mictc_set_win(int on);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_CTC_H_ */
