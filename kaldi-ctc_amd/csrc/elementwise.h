// elementwise.h -- small bandwidth-bound kernels of the train step.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace kctc {

// w += lr * clamp(dw, -clip, clip)   (clip <= 0: no clamp).  skip (device,
// nullable): when *skip != 0 the update is not applied (a failed step).
void clip_sgd_update(hipStream_t s, float *w, const float *dw, long n, float lr, float clip,
                     const unsigned *skip = nullptr);
// momentum form (TrainNnetSimple with a delta nnet, ctc-nnet-train.cc:194-245):
// delta += lr * clamp(dw); w += delta; delta *= m
void momentum_update(hipStream_t s, float *w, float *delta, const float *dw, long n, float lr, float clip,
                     float m, const unsigned *skip = nullptr);
// ClipGradientComponent norm-based backprop: rows with |row| >= thr scaled to
// norm thr; *nclipped (device int) += number of such rows.
void rownorm_clip(hipStream_t s, float *d, long rows, int dim, float thr, int *nclipped);
// best-path ids: _find_row_max_id tie rule (-1 when nothing > -1e20)
void row_argmax(hipStream_t s, const float *m, long rows, int cols, int *ids);
// out[j] = alpha * sum_rows X[:, j] + beta * out[j]; ws >= sum_rows_ws_floats
size_t sum_rows_ws_floats(long rows, int cols);
void sum_rows(hipStream_t s, const float *X, long rows, int cols, float alpha, float beta,
              float *out, float *ws);
void fill(hipStream_t s, float *p, long n, float v);
void scale_inplace(hipStream_t s, float *p, long n, float alpha);
// y += alpha * x (CuVector::AddVec)
void axpy(hipStream_t s, float *y, const float *x, long n, float alpha);
// x += stddev * N(0,1) (PerturbParams: a temporary SetRandn() then AddVec);
// element i draws from a counter-based splitmix64 + Box-Muller stream of
// (seed, i), so the noise does not depend on the launch shape
void add_randn(hipStream_t s, float *x, long n, float stddev, unsigned long long seed);
// *out (device double) = sum_i a[i] * b[i] (VecVec / TraceMatMat over the flat
// parameters), fp64 accumulation in a fixed order: deterministic
size_t dot_ws_bytes();
void dot_f64(hipStream_t s, const float *a, const float *b, long n, double *out, void *ws);

// SpliceComponent on the FormatNnetInput layout (nnet.h): output row j, block
// c = input row j * ns + first + ctx[c] (dim - const_dim columns); the last
// const_dim columns from input row j * ns.  Backward: the transpose (input
// rows no block reads get zeros; the const part adds to the chunk's first
// row).  At most kMaxSplice context offsets.
constexpr int kMaxSplice = 32;
void splice_rows(hipStream_t s, const float *in, int dim, int ns, long rows, const int *ctx, int nctx, int first,
                 int const_dim, float *out);
void splice_rows_backward(hipStream_t s, const float *out_deriv, int dim, int ns, long rows, const int *ctx, int nctx,
                          int first, int const_dim, float *in_deriv);

// NnetComputer's padded input (nnet-compute.cc:64-90, pad = true) laid out
// for this path's SpliceComponent (ns = 1 + left + right rows per output
// frame): out row t*ns + s = feats row clamp(t + s - left, 0, T-1) (the first
// and last frames repeated left / right times), feats [T][dim] -> out [T*ns][dim]
void pad_splice_input(hipStream_t s, const float *feats, int T, int dim, int left, int ns, float *out);

// Data-parallel agreement on a failed step: the step's device error word (set
// by a recurrence's bounded-spin timeout) as a 0/1 float that the gradient
// exchange sums over the ranks, and back: a positive sum sets kErrPeerFailed,
// so every rank skips the updates of a step that failed on any rank.
constexpr unsigned kErrPeerFailed = 1u << 8;
void err_word_to_flag(hipStream_t s, const unsigned *err, float *flag);
void flag_to_err_word(hipStream_t s, const float *flag, unsigned *err);

// Holds `blocks` whole CUs (1024 threads and 160 KB LDS each) for `usec`
// microseconds: the stand-in for a communication kernel in the CU-budget test.
void cu_hold(hipStream_t s, int blocks, double usec);
// Where the blocks of a launch on `s` run: `blocks` blocks, each ~usec long,
// write (XCC_ID << 16) | (HW_ID bits 8..15: CU, SH, SE) into ids[block].
void cu_where(hipStream_t s, unsigned *ids, int blocks, double usec);

}  // namespace kctc
