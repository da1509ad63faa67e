// cumatrix_api.cpp -- C ABI of include/kaldi_cumatrix.h.
#include "kaldi_cumatrix.h"

#include <algorithm>

#include "common.h"
#include "elementwise.h"
#include "gemm.h"

extern "C" {

int kcm_add_mat_mat(struct ihipStream_t *stream, int transA, int transB, int M, int N, int K,
                    float alpha, const float *A, long lda, const float *B, long ldb, float beta,
                    float *C, long ldc) {
  if (M < 0 || N < 0 || K < 0 || !C) return 1;
  try {
    kctc::GemmArgs g;
    g.transA = transA != 0; g.transB = transB != 0;
    g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
    g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
    kctc::gemm_f32(stream, g);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  } catch (...) {
    return 3;
  }
}

size_t kcm_add_mat_mat_x3_workspace(int M, int N, int K) {
  if (M < 0 || N < 0 || K < 0) return 0;
  return kctc::align_up(kctc::x3p_bytes(M, K), 256) + kctc::align_up(kctc::x3p_bytes(N, K), 256) +
         sizeof(int) * (size_t)(M + N) + sizeof(unsigned) * (size_t)std::max(M, N) + 256;
}

int kcm_add_mat_mat_x3(struct ihipStream_t *stream, int transA, int transB, int M, int N, int K,
                       float alpha, const float *A, long lda, const float *B, long ldb, float beta,
                       float *C, long ldc, void *ws) {
  if (M < 0 || N < 0 || K < 0 || !C || !ws) return 1;
  try {
    char *w = static_cast<char *>(ws);
    _Float16 *Ap = reinterpret_cast<_Float16 *>(w);
    w += kctc::align_up(kctc::x3p_bytes(M, K), 256);
    _Float16 *Bp = reinterpret_cast<_Float16 *>(w);
    w += kctc::align_up(kctc::x3p_bytes(N, K), 256);
    int *eA = reinterpret_cast<int *>(w);
    int *eB = eA + M;
    unsigned *cm = reinterpret_cast<unsigned *>(eB + N);
    // op(A) rows: rows of A (M x K) or columns of A^T (K x M)
    if (!transA) {
      kctc::x3p_pack_rows(stream, A, lda, M, K, Ap, eA, 0.f);
    } else {
      kctc::absmax_f32(stream, A, lda, K, M, nullptr, cm);
      kctc::x3p_pack_cols(stream, A, lda, K, M, 0, Ap, eA, cm, 0.f);
    }
    // op(B) columns: rows of B^T (N x K) or columns of B (K x N)
    if (transB) {
      kctc::x3p_pack_rows(stream, B, ldb, N, K, Bp, eB, 0.f);
    } else {
      kctc::absmax_f32(stream, B, ldb, K, N, nullptr, cm);
      kctc::x3p_pack_cols(stream, B, ldb, K, N, 0, Bp, eB, cm, 0.f);
    }
    kctc::X3PArgs g;
    g.M = M; g.N = N; g.KB = (K + 31) / 32;
    g.A = Ap; g.B = Bp; g.eA = eA; g.eB = eB;
    g.C = C; g.ldc = ldc; g.alpha = alpha; g.beta = beta;
    kctc::gemm_x3p(stream, g);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  } catch (...) {
    return 3;
  }
}

int kcm_find_row_max_id(struct ihipStream_t *stream, const float *m, long rows, int cols, int *ids) {
  if (!m || !ids || cols <= 0) return 1;
  kctc::row_argmax(stream, m, rows, cols, ids);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int kcm_clip_gradient_rows(struct ihipStream_t *stream, float *deriv, long rows, int dim,
                           float threshold, int *num_clipped_dev) {
  if (!deriv || !num_clipped_dev || dim <= 0 || !(threshold > 0.f)) return 1;
  kctc::rownorm_clip(stream, deriv, rows, dim, threshold, num_clipped_dev);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int kcm_add_vec_clipped(struct ihipStream_t *stream, float *w, const float *dw, long n, float lr,
                        float clip) {
  if (!w || !dw) return 1;
  kctc::clip_sgd_update(stream, w, dw, n, lr, clip);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int kcm_add_row_sum_mat(struct ihipStream_t *stream, const float *X, long rows, int cols,
                        float alpha, float beta, float *out, float *ws) {
  if (!X || !out || !ws) return 1;
  kctc::sum_rows(stream, X, rows, cols, alpha, beta, out, ws);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
