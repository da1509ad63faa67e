/*
 * kaldi_cumatrix.h -- the CuMatrix/CuVector operations the CTC-train path
 * touches, as a row-major C ABI over gfx950 kernels
 * (gemm.hip, elementwise.hip).  All calls are ordered on `stream` and never
 * synchronise the host.  Return 0 on success.
 */
#ifndef KALDI_CTC_AMD_KALDI_CUMATRIX_H_
#define KALDI_CTC_AMD_KALDI_CUMATRIX_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;

/* C = alpha op(A) op(B) + beta C, row-major, fp32 MFMA.  Replaces
 * CuMatrixBase::AddMatMat -> cublasSgemm (src/cudamatrix/cu-matrix.cc:1077-1110)
 * as used by AffineComponent (src/nnet2/nnet-component.cc:1184-1226). */
int kcm_add_mat_mat(struct ihipStream_t *stream, int transA, int transB, int M, int N, int K,
                    float alpha, const float *A, long lda, const float *B, long ldb, float beta,
                    float *C, long ldc);
/* The same product on the split-fp16 matrix-core path (fp32-class: every row
 * of op(A) and column of op(B) is scaled by a power of two and carried as an
 * fp16 hi + lo pair, hi*hi + hi*lo + lo*hi accumulated in fp32; both operands
 * are first packed along K, gemm_x3p.hip).  ws: device scratch of at least
 * kcm_add_mat_mat_x3_workspace(M, N, K) bytes. */
size_t kcm_add_mat_mat_x3_workspace(int M, int N, int K);
int kcm_add_mat_mat_x3(struct ihipStream_t *stream, int transA, int transB, int M, int N, int K,
                       float alpha, const float *A, long lda, const float *B, long ldb, float beta,
                       float *C, long ldc, void *ws);
/* ids[r] = argmax_c m[r][c].  Replaces CuMatrix::FindRowMaxId on the device
 * (src/cudamatrix/cu-matrix.cc:1612-1628 -> _find_row_max_id,
 * src/cudamatrix/cu-kernels.cu:2454-2500) with the same result bit for bit:
 * only values > -1e20 count (else -1), and ties resolve as that kernel's
 * 256-thread strict-greater reduction tree does (not always to the lowest
 * column; equal maxima at columns 1 and 2 give 2). */
int kcm_find_row_max_id(struct ihipStream_t *stream, const float *m, long rows, int cols, int *ids);
/* ClipGradientComponent norm-based backprop (src/nnet2/nnet-cudnn-component.cc:936-957):
 * rows with |row|_2 >= threshold rescaled to norm threshold; *num_clipped_dev
 * (device int) += number of such rows. */
int kcm_clip_gradient_rows(struct ihipStream_t *stream, float *deriv, long rows, int dim,
                           float threshold, int *num_clipped_dev);
/* w += lr * clamp(dw, -clip, clip) (clip <= 0: no clamp).  Replaces
 * ApplyFloor/ApplyCeiling + AddVec (nnet-cudnn-component.cc:602-614). */
int kcm_add_vec_clipped(struct ihipStream_t *stream, float *w, const float *dw, long n, float lr,
                        float clip);
/* out = alpha * (sum of the rows of X) + beta * out.  Replaces CuVector::AddRowSumMat
 * (src/cudamatrix/cu-vector.cc:1157-1165).  ws: >= 64*cols floats of device scratch. */
int kcm_add_row_sum_mat(struct ihipStream_t *stream, const float *X, long rows, int cols,
                        float alpha, float beta, float *out, float *ws);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_KALDI_CUMATRIX_H_ */
