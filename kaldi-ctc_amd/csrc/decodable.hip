// decodable.hip -- the decode-side use of a trained CTC model (SURVEY §8f
// row 3): SoftmaxComponent::Propagate (the component the recipe appends
// before decoding, egs/wsj/s5/steps/ctc/train.sh:471-477) and the
// CtcDecodableAmNnet log-likelihood matrix (src/ctc/ctc-decodable-am-nnet.cc:28-80):
//
//   probs = softmax(nnet output), floored at 1e-20     (nnet-component.cc:929-946)
//   if blank_threshold < 1: keep only frames with probs[t][0] < blank_threshold
//     (all of them if none would remain)               (:52-68)
//   log_probs = log(max(probs, floor))                 (:70-71, floor 1e-10;
//                                                       CtcDecodableAmNnetParallel 1e-20)
//   log_probs -= log(priors)   (when the AmNnet has priors)  (:73-79)
//   log_probs *= prob_scale                            (:81-82)
//
// Kernels: k_softmax_rows (one wave per row), k_blank_scan (one workgroup:
// ordered compaction of the kept frames, the CopyRows of :63-65), and
// k_decodable_rows (one wave per kept row: gather, floor, log, prior, scale).
#include "common.h"
#include "decodable.h"

namespace kctc {
namespace {

__global__ __launch_bounds__(256) void k_softmax_rows(const float *__restrict__ in, long rows, int cols,
                                                      float *__restrict__ out) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float *x = in + row * cols;
  float m = -INFINITY;
  for (int j = lane; j < cols; j += 64) m = fmaxf(m, x[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) s += expf(x[j] - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  float *y = out + row * cols;
  for (int j = lane; j < cols; j += 64) y[j] = fmaxf(expf(x[j] - m) * inv, 1.0e-20f);
}

// dst[t] = index of frame t among the kept frames (or -1); *kept = count.
// One workgroup scans the T flags in chunks of 1024 in frame order.
__global__ __launch_bounds__(1024) void k_blank_scan(const float *__restrict__ probs, int T, int A,
                                                     float blank_threshold, int *__restrict__ dst,
                                                     int *__restrict__ kept) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool skip = blank_threshold < 1.0f;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < T; c0 += 1024) {
    const int t = c0 + tid;
    const int k = (t < T) && (!skip || probs[(long)t * A] < blank_threshold) ? 1 : 0;
    // inclusive scan within the wave, then across the 16 waves
    int v = k;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    int off = base;
    for (int i = 0; i < w; i++) off += wsum[i];
    if (t < T) dst[t] = k ? off + v - 1 : -1;
    __syncthreads();
    if (tid == 1023) base = off + v;
    __syncthreads();
  }
  // "No Frame will be keeped ..., don't skip blank" (:59-61)
  const bool none = skip && base == 0;
  if (none)
    for (int t = tid; t < T; t += 1024) dst[t] = t;
  if (tid == 0) *kept = none ? T : base;
}

__global__ __launch_bounds__(256) void k_decodable_rows(const float *__restrict__ probs, int T, int A,
                                                        const int *__restrict__ dst,
                                                        const float *__restrict__ priors, float prob_scale,
                                                        float floor_v, float *__restrict__ out) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const int r = dst[t];
  if (r < 0) return;
  const float *p = probs + (long)t * A;
  float *o = out + (long)r * A;
  for (int j = lane; j < A; j += 64) {
    float v = logf(fmaxf(p[j], floor_v));          // ApplyFloor, ApplyLog
    if (priors) v += -1.0f * logf(priors[j]);      // AddVecToRows(-1.0, log priors)
    o[j] = v * prob_scale;                         // Scale(prob_scale)
  }
}

// DiffSoftmaxPerRow (SoftmaxComponent::Backprop, nnet-component.cc:948-976):
// d_i = p_i e_i - p_i (p . e), one wave per row
__global__ __launch_bounds__(256) void k_diff_softmax_rows(const float *__restrict__ p, const float *__restrict__ e,
                                                           long rows, int cols, float *__restrict__ d) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float *pr = p + row * cols, *er = e + row * cols;
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) s += pr[j] * er[j];
  s = wave_sum(s);
  float *dr = d + row * cols;
  for (int j = lane; j < cols; j += 64) dr[j] = pr[j] * (er[j] - s);
}

}  // namespace

void diff_softmax_rows(hipStream_t s, const float *value, const float *deriv, long rows, int cols, float *out) {
  if (rows <= 0 || cols <= 0) return;
  hipLaunchKernelGGL(k_diff_softmax_rows, dim3(ceil_div(rows, 4)), dim3(256), 0, s, value, deriv, rows, cols, out);
}

void softmax_rows(hipStream_t s, const float *in, long rows, int cols, float *out) {
  if (rows <= 0 || cols <= 0) return;
  hipLaunchKernelGGL(k_softmax_rows, dim3(ceil_div(rows, 4)), dim3(256), 0, s, in, rows, cols, out);
}

size_t ctc_decodable_scratch_bytes(int T) { return sizeof(int) * ((size_t)T + 64); }

void ctc_decodable(hipStream_t s, const float *probs, int T, int A, const float *priors, float prob_scale,
                   float blank_threshold, float floor_v, float *out, void *scratch, int *kept_dev) {
  if (T <= 0 || A <= 0) return;
  int *dst = static_cast<int *>(scratch);
  hipLaunchKernelGGL(k_blank_scan, dim3(1), dim3(1024), 0, s, probs, T, A, blank_threshold, dst, kept_dev);
  hipLaunchKernelGGL(k_decodable_rows, dim3(ceil_div(T, 4)), dim3(256), 0, s, probs, T, A, dst, priors, prob_scale,
                     floor_v, out);
}

}  // namespace kctc
