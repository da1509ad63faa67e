// clipgrad.hip -- ClipGradientComponent::Backprop + RepairGradients on device
// (reference src/nnet2/nnet-cudnn-component.cc:921-1055).
//
// The reference decides the self-repair on the host after reading back the
// clip count (a D2H sync per component per minibatch).  Here every scalar
// stays on the device: the cumulative counters live in a small DevState, the
// repair kernels read the proportion and gate themselves.  Only the
// RandUniform() draw (host RNG) is decided on the host, exactly where the
// reference draws it.  Sums over rows are two-stage and fixed-order
// (deterministic).
#include "clipgrad.h"
#include "common.h"
#include "elementwise.h"

namespace kctc {
namespace {

using State = ClipState;

__global__ void k_commit(State *st, long rows) {
  st->num_clipped += (double)st->step_clipped;
  st->count += (double)rows;
  st->step_clipped = 0;
}

__global__ __launch_bounds__(256) void k_clamp(float *d, long n, float thr) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    d[i] = fminf(fmaxf(d[i], -thr), thr);
}

__device__ __forceinline__ float repair_val(float x, float target) {
  const float sgn = x > 0.f ? 1.f : -1.f;  // ApplyHeaviside*2-1: x<=0 -> -1
  const float m = fabsf(x) - target;
  return (m > 0.f ? m : 0.f) * sgn;
}

// one wave per row: ||d_row||, ||repair_row||  -> per-block partials (double)
__global__ __launch_bounds__(256) void k_norms(const float *__restrict__ d, const float *__restrict__ x,
                                               long rows, int dim, float target, int with_rep,
                                               double *__restrict__ part) {
  __shared__ double sh[2][4];
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float a = 0.f, b = 0.f;
  if (row < rows) {
    for (int j = lane; j < dim; j += 64) {
      const float v = d[row * dim + j];
      a += v * v;
      if (with_rep) {
        const float r = repair_val(x[row * dim + j], target);
        b += r * r;
      }
    }
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    sh[0][w] = row < rows ? sqrt((double)a) : 0.0;
    sh[1][w] = row < rows ? sqrt((double)b) : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ((sh[0][0] + sh[0][1]) + sh[0][2]) + sh[0][3];
    part[2 * blockIdx.x + 1] = ((sh[1][0] + sh[1][1]) + sh[1][2]) + sh[1][3];
  }
}

__device__ double block_sum(double v) {
  __shared__ double sh[4];
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = ((sh[0] + sh[1]) + sh[2]) + sh[3];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_decide(State *st, const State *dec, const double *__restrict__ part,
                                                int nb, long rows, float threshold, float scale) {
  double a = 0, b = 0;
  for (int i = threadIdx.x; i < nb; i += 256) { a += part[2 * i]; b += part[2 * i + 1]; }
  a = block_sum(a);
  b = block_sum(b);
  if (threadIdx.x == 0) {
    const double prop = dec->count > 0 ? dec->num_clipped / dec->count : 0.0;
    st->active = prop > (double)threshold;
    st->dn = a;
    st->rn = b;
    st->scale = 0.0;
    if (st->active) {
      st->num_self_repaired += 1.0;
      const double magnitude = (double)scale * prop * (a / (double)rows);
      const double s = b != 0.0 ? magnitude / (b / (double)rows) : 0.0;
      st->scale = -s / 0.5;  // repair_probability = 0.5
    }
  }
}

__global__ __launch_bounds__(256) void k_apply(float *__restrict__ d, const float *__restrict__ x,
                                               long rows, int dim, float target, const State *st,
                                               double *__restrict__ part) {
  __shared__ double sh[4];
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool active = st->active;
  const float alpha = (float)st->scale;
  float a = 0.f;
  if (active && row < rows) {
    for (int j = lane; j < dim; j += 64) {
      float v = d[row * dim + j] + alpha * repair_val(x[row * dim + j], target);
      d[row * dim + j] = v;
      a += v * v;
    }
  }
  a = wave_sum(a);
  if (lane == 0) sh[w] = row < rows ? sqrt((double)a) : 0.0;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

__global__ __launch_bounds__(256) void k_final(State *st, const double *__restrict__ part, int nb) {
  double a = 0;
  for (int i = threadIdx.x; i < nb; i += 256) a += part[i];
  a = block_sum(a);
  if (threadIdx.x == 0) st->dn2 = (st->active && a != 0.0) ? st->dn / a : 1.0;
}

__global__ __launch_bounds__(256) void k_rescale(float *d, long n, const State *st) {
  if (!st->active) return;
  const float f = (float)st->dn2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) d[i] *= f;
}

}  // namespace

size_t clipgrad_scratch_bytes(long rows) { return sizeof(double) * 2 * (size_t)(rows / 4 + 2); }

void clipgrad_backprop(hipStream_t s, float *d, const float *in_value, long rows, int dim,
                       float threshold, bool norm_based, bool try_repair, float repair_threshold,
                       float repair_target, float repair_scale, ClipState *st, void *scratch,
                       const ClipState *decide) {
  if (!decide) decide = st;
  if (rows <= 0 || !(threshold > 0.f)) return;
  if (norm_based) {
    rownorm_clip(s, d, rows, dim, threshold, &st->step_clipped);
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, s, st, rows);
  } else {
    const long n = rows * (long)dim;
    hipLaunchKernelGGL(k_clamp, dim3((int)std::min<long>(4096, (n + 255) / 256)), dim3(256), 0, s, d,
                       n, threshold);
  }
  if (!try_repair) return;
  double *part = static_cast<double *>(scratch);
  const int nb = ceil_div(rows, 4);
  hipLaunchKernelGGL(k_norms, dim3(nb), dim3(256), 0, s, d, in_value, rows, dim, repair_target, 1,
                     part);
  hipLaunchKernelGGL(k_decide, dim3(1), dim3(256), 0, s, st, decide, part, nb, rows,
                     repair_threshold, repair_scale);
  hipLaunchKernelGGL(k_apply, dim3(nb), dim3(256), 0, s, d, in_value, rows, dim, repair_target, st,
                     part);
  hipLaunchKernelGGL(k_final, dim3(1), dim3(256), 0, s, st, part, nb);
  const long n = rows * (long)dim;
  hipLaunchKernelGGL(k_rescale, dim3((int)std::min<long>(4096, (n + 255) / 256)), dim3(256), 0, s,
                     d, n, st);
}

}  // namespace kctc
