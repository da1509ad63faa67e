/*
 * test_hooks.h -- measurement and test entry points of libkaldictc_amd.so
 * that have no reference counterpart and are not part of the drop-in ABI
 * (the headers under include/).  Used only by tests/, bench.py and scripts/.
 */
#ifndef KALDI_CTC_AMD_TEST_HOOKS_H_
#define KALDI_CTC_AMD_TEST_HOOKS_H_

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;

/* Average ms of the packed gate GEMM (the kernel under kcm_add_mat_mat_x3
 * and the RNN GEMMs) on random packed operands, C[M][N] = A[M][K] B[N][K]^T, split-fp16 (bf16 = 0) or bf16
 * operands, split-K slices; -1 on failure. */
float kcm_bench_gemm_packed(struct ihipStream_t *stream, int M, int N, int K, int bf16, int iters, int split);
/* The streamed direction-split GEMM of the RNN backward (dx) and chained forward (next projection) against a
 * producer that has already finished: C[M][N] = E[:, 0:K] Wt[0]^T +
 * E[:, K:2K] Wt[1]^T (+ bias[c]), E [M][2K], Wt [2][N][K], device pointers;
 * forward: the producer's direction order of a forward recurrence; tail_rows:
 * split-K tail slots per direction (-1: default).  1 on unsupported shapes. */
int kcm_test_row_stream(struct ihipStream_t *stream, int M, int N, int K, int forward, int tail_rows,
                        const float *E, const float *Wt, const float *bias, float *C);
/* A CuDNNRecurrentComponent handle (include/kaldi_nnet2_component.h) with
 * the trainer's side streams and forward-time prepacks on (on = 1): its
 * Propagate packs W^T and x^T / y^T beside the recurrence, its Backprop
 * streams dx and runs the weight GEMMs on the side stream, as in training. */
struct kctcComponentImpl;
int kctc_test_component_side_streams(struct kctcComponentImpl *h, int on);
#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_TEST_HOOKS_H_ */
