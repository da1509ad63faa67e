// gemm.h -- fp32 MFMA GEMM for gfx950 (v_mfma_f32_16x16x4_f32, exact fp32).
// Replaces the cublasSgemm calls of the reference's CuMatrix::AddMatMat
// (src/cudamatrix/cu-matrix.cc:1077-1110) and cuDNN's internal gate GEMMs.
#pragma once
#include <hip/hip_runtime.h>

namespace kctc {

// Row-major: C[b][i][j] = alpha * sum_k opA(b,i,k) opB(b,k,j) + beta * C[b][i][j]
//                         (+ bias[b][j] + bias2[b][j] when given)
//   opA(i,k) = transA ? A[k*lda + i] : A[i*lda + k]
//   opB(k,j) = transB ? B[j*ldb + k] : B[k*ldb + j]
// Batch strides may be negative.  split_k > 1 needs `ws` of
// split_k * batch * M * N floats and makes the result deterministic (slab
// reduce in fixed order).
struct GemmArgs {
  bool transA = false, transB = false;
  int M = 0, N = 0, K = 0;
  float alpha = 1.f, beta = 0.f;
  const float *A = nullptr, *B = nullptr;
  float *C = nullptr;
  long lda = 0, ldb = 0, ldc = 0;
  const float *bias = nullptr, *bias2 = nullptr;
  int batch = 1;
  long strideA = 0, strideB = 0, strideC = 0, strideBias = 0;
  int split_k = 1;
  float *ws = nullptr;
  int max_blocks = 0;  // > 0: persistent grid of at most this many workgroups
  // optional: zeroed device int -> dynamic tile scheduling (blocks pull work
  // items from this counter; blocks that start late, e.g. on CUs a concurrent
  // persistent kernel holds, find the work done and exit)
  int *tile_counter = nullptr;
};

void gemm_f32(hipStream_t stream, const GemmArgs &g);
// Heuristic split-K so that tiles * split fill the chip; returns 1 if not needed.
int gemm_pick_split(int M, int N, int K, int batch);

// Split-fp16 ("x3") GEMM, same contract as gemm_f32 (fp32-class results, see
// gemm.hip).  Operand scaling: per A row (M index) / per B column (N index)
// max |x| as float bits (absmax_f32), or, when the array is null, a constant
// bound on |x| (e.g. 1 for an LSTM/GRU output).
struct X3Scales {
  const unsigned *amaxA = nullptr, *amaxB = nullptr;
  long strideA = 0, strideB = 0;  // per batch
  float boundA = 1.f, boundB = 1.f;
};
void gemm_x3(hipStream_t stream, const GemmArgs &g, const X3Scales &s);
int split_exp_host(float bound);
// max |X| per row (rmax[b][r]) and per column (cmax[b][c]) as float bits; either may be null
void absmax_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, unsigned *rmax, unsigned *cmax,
                int batch = 1, long strideX = 0, long strideR = 0, long strideC = 0);

// column sums: out[b][j] (+)= alpha * sum_i X[b][i*ldx + j], i < rows  (accumulate if beta=1)
void colsum_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, float alpha,
                float beta, float *out, int batch = 1, long strideX = 0, long strideOut = 0);

}  // namespace kctc
