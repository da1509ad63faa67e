// elementwise.hip -- the small bandwidth-bound kernels of the train step.
// They replace the CuVector/CuMatrix ops the reference touches on this path
// (SURVEY.md §2.2): _vec_apply_floor/_ceiling + cublas axpy (dW clip and SGD,
// nnet-cudnn-component.cc:602-614), the ClipGradientComponent row-norm clip
// (AddDiagMat2 / ApplyFloor / ApplyPow / MulRowsVec, :921-970) and
// _find_row_max_id (cu-kernels.cu:2454-2500).  All loads/stores are 16-B
// vectorised where the row layout allows; no host synchronisation.
#include "common.h"
#include "elementwise.h"

namespace kctc {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_clip_sgd(float *__restrict__ w, const float *__restrict__ dw,
                                                  long n, float lr, float clip, const unsigned *skip) {
  if (skip && *skip) return;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * 256;
  const bool vec = ((uintptr_t)w % 16 == 0) && ((uintptr_t)dw % 16 == 0);
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (vec) {
    for (; i < n4; i += stride) {
      floatx4 g = reinterpret_cast<const floatx4 *>(dw)[i];
      floatx4 v = reinterpret_cast<floatx4 *>(w)[i];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        float x = g[j];
        if (clip > 0.f) x = fminf(fmaxf(x, -clip), clip);
        v[j] += lr * x;
      }
      reinterpret_cast<floatx4 *>(w)[i] = v;
    }
    i = n4 * 4 + (long)blockIdx.x * 256 + threadIdx.x;
  }
  for (; i < n; i += stride) {
    float x = dw[i];
    if (clip > 0.f) x = fminf(fmaxf(x, -clip), clip);
    w[i] += lr * x;
  }
}

// One wave per row: scale = (|row|^2/thr^2 < 1) ? 1 : rsqrt(|row|^2/thr^2)
__global__ __launch_bounds__(256) void k_rownorm_clip(float *__restrict__ d, long rows, int dim,
                                                      float inv_thr2, int *__restrict__ nclipped) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ int cnt[4];
  int clipped = 0;
  if (row < rows) {
    float *r = d + row * dim;
    float ss = 0.f;
    const bool vec = (dim % 4 == 0) && ((uintptr_t)r % 16 == 0);
    if (vec) {
      for (int j = lane; j < dim / 4; j += 64) {
        floatx4 v = reinterpret_cast<const floatx4 *>(r)[j];
        ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      }
    } else {
      for (int j = lane; j < dim; j += 64) ss += r[j] * r[j];
    }
    ss = wave_sum(ss);
    const float sc = ss * inv_thr2;
    if (!(sc < 1.f)) {
      clipped = 1;
      const float f = rsqrtf(sc);
      if (vec) {
        for (int j = lane; j < dim / 4; j += 64) {
          floatx4 v = reinterpret_cast<const floatx4 *>(r)[j];
          reinterpret_cast<floatx4 *>(r)[j] = v * f;
        }
      } else {
        for (int j = lane; j < dim; j += 64) r[j] *= f;
      }
    }
  }
  if (lane == 0) cnt[threadIdx.x >> 6] = clipped;
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = cnt[0] + cnt[1] + cnt[2] + cnt[3];
    if (c) atomicAdd(nclipped, c);
  }
}

// FindRowMaxId with the tie rule of the kernel the reference's CTC path runs,
// _find_row_max_id (cu-kernels.cu:2454-2500): 256 virtual threads t keep the
// first strict maximum above -1e20f of columns t, t+256, ...; a tree then lets
// position p take p+w (w = 128 .. 1) only when strictly greater, so ties
// resolve by the tree position, and a row with nothing above -1e20 gives -1.
// Here one wave per row: lane l holds virtual threads l, l+64, l+128, l+192;
// levels 128 and 64 combine in registers, 32 .. 1 by shuffles (a lane reads its
// source's value from before the level, as the tree does).
__global__ __launch_bounds__(256) void k_row_argmax(const float *__restrict__ m, long rows, int cols,
                                                    int *__restrict__ ids) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float *r = m + row * cols;
  float v[4];
  int vi[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k] = -1e20f;
    vi[k] = -1;
    for (int j = lane + 64 * k; j < cols; j += 256) {
      const float x = r[j];
      if (x > v[k]) { v[k] = x; vi[k] = j; }
    }
  }
  if (v[2] > v[0]) { v[0] = v[2]; vi[0] = vi[2]; }  // w = 128
  if (v[3] > v[1]) { v[1] = v[3]; vi[1] = vi[3]; }
  if (v[1] > v[0]) { v[0] = v[1]; vi[0] = vi[1]; }  // w = 64
  float b = v[0];
  int bi = vi[0];
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const float ob = __shfl_down(b, w, 64);
    const int oi = __shfl_down(bi, w, 64);
    if (ob > b) { b = ob; bi = oi; }
  }
  if (lane == 0) ids[row] = bi;
}

// out[j] = alpha * sum_i X[i][j] + beta * out[j]; one workgroup per 64 cols,
// rows split over 4 wave groups, combined in a fixed order (deterministic).
__global__ __launch_bounds__(256) void k_sum_rows(const float *__restrict__ X, long rows, int cols,
                                                  float alpha, float beta, float *__restrict__ out) {
  __shared__ float part[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  float s = 0.f;
  if (c < cols)
    for (long r = blockIdx.y * 4 + g; r < rows; r += 4L * gridDim.y) s += X[r * cols + c];
  part[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < cols) {
    float v = ((part[0][threadIdx.x] + part[1][threadIdx.x]) + part[2][threadIdx.x]) + part[3][threadIdx.x];
    out[(long)blockIdx.y * cols + c] = v;
  }
}

__global__ __launch_bounds__(256) void k_sum_partials(const float *__restrict__ part, int nparts,
                                                      int cols, float alpha, float beta,
                                                      float *__restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int p = 0; p < nparts; p++) s += part[(long)p * cols + c];
  out[c] = alpha * s + (beta != 0.f ? beta * out[c] : 0.f);
}

__global__ void k_scale(float *p, long n, float a) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] *= a;
}

__global__ void k_fill(float *p, long n, float v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = v;
}

}  // namespace

static int grid_for(long n, int per = 256) {
  long b = (n + per - 1) / per;
  return (int)std::max<long>(1, std::min<long>(b, 4096));
}

__global__ __launch_bounds__(256) void k_momentum(float *__restrict__ w, float *__restrict__ delta,
                                                  const float *__restrict__ dw, long n, float lr, float clip,
                                                  float m, const unsigned *skip) {
  if (skip && *skip) return;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float g = dw[i];
    if (clip > 0.f) g = fminf(fmaxf(g, -clip), clip);
    const float dl = delta[i] + lr * g;
    w[i] += dl;
    delta[i] = m * dl;
  }
}

void momentum_update(hipStream_t s, float *w, float *delta, const float *dw, long n, float lr, float clip,
                     float m, const unsigned *skip) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_momentum, dim3(grid_for(n)), dim3(256), 0, s, w, delta, dw, n, lr, clip, m, skip);
}

void clip_sgd_update(hipStream_t s, float *w, const float *dw, long n, float lr, float clip,
                     const unsigned *skip) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_clip_sgd, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, w, dw, n, lr, clip, skip);
}

void rownorm_clip(hipStream_t s, float *d, long rows, int dim, float thr, int *nclipped) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_rownorm_clip, dim3(ceil_div(rows, 4)), dim3(256), 0, s, d, rows, dim,
                     1.f / (thr * thr), nclipped);
}

void row_argmax(hipStream_t s, const float *m, long rows, int cols, int *ids) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_row_argmax, dim3(ceil_div(rows, 4)), dim3(256), 0, s, m, rows, cols, ids);
}

size_t sum_rows_ws_floats(long rows, int cols) { return (size_t)64 * cols; }

void sum_rows(hipStream_t s, const float *X, long rows, int cols, float alpha, float beta,
              float *out, float *ws) {
  if (cols <= 0) return;
  const int parts = (int)std::min<long>(64, std::max<long>(1, rows / 256));
  hipLaunchKernelGGL(k_sum_rows, dim3(ceil_div(cols, 64), parts), dim3(256), 0, s, X, rows, cols,
                     alpha, beta, ws);
  hipLaunchKernelGGL(k_sum_partials, dim3(ceil_div(cols, 256)), dim3(256), 0, s, ws, parts, cols,
                     alpha, beta, out);
}

void fill(hipStream_t s, float *p, long n, float v) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(256), 0, s, p, n, v);
}

void scale_inplace(hipStream_t s, float *p, long n, float alpha) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(256), 0, s, p, n, alpha);
}

// ---- UpdatableComponent parameter arithmetic --------------------------------
__global__ void k_axpy(float *__restrict__ y, const float *__restrict__ x, long n, float a) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] += a * x[i];
}

__device__ __forceinline__ unsigned long long splitmix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ void k_add_randn(float *__restrict__ x, long n, float stddev, unsigned long long seed) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned long long a = splitmix(seed ^ splitmix(2ull * (unsigned long long)i));
    const unsigned long long b = splitmix(seed ^ splitmix(2ull * (unsigned long long)i + 1ull));
    const double u1 = ((double)(a >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    const double u2 = ((double)(b >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    x[i] += stddev * (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
  }
}

constexpr int kDotBlocks = 256;
// fixed grid: block b sums elements b*256+tid, + kDotBlocks*256, ... in fp64,
// then a fixed-order tree; the partials are summed in block order
__global__ __launch_bounds__(256) void k_dot_partial(const float *__restrict__ a, const float *__restrict__ b,
                                                     long n, double *__restrict__ part) {
  __shared__ double w[4];
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)kDotBlocks * 256)
    s += (double)a[i] * (double)b[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}
__global__ __launch_bounds__(64) void k_dot_final(const double *__restrict__ part, double *__restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < kDotBlocks; i += 64) s += part[i];
  s = wave_sum_d(s);
  if (threadIdx.x == 0) *out = s;
}

void axpy(hipStream_t s, float *y, const float *x, long n, float alpha) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n)), dim3(256), 0, s, y, x, n, alpha);
}

void add_randn(hipStream_t s, float *x, long n, float stddev, unsigned long long seed) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_add_randn, dim3(grid_for(n)), dim3(256), 0, s, x, n, stddev, seed);
}

size_t dot_ws_bytes() { return sizeof(double) * kDotBlocks; }

void dot_f64(hipStream_t s, const float *a, const float *b, long n, double *out, void *ws) {
  double *part = static_cast<double *>(ws);
  hipLaunchKernelGGL(k_dot_partial, dim3(kDotBlocks), dim3(256), 0, s, a, b, n < 0 ? 0 : n, part);
  hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(64), 0, s, part, out);
}

// ---- SpliceComponent --------------------------------------------------------
struct SpliceArgs {
  int n, first, dim, const_dim, ns, out_dim;
  int ctx[kMaxSplice];
};
// one thread per output element; rows of the same chunk are contiguous
__global__ void k_splice(const float *__restrict__ in, long rows, SpliceArgs a, float *__restrict__ out) {
  const long total = rows * a.out_dim;
  const int sd = a.dim - a.const_dim;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long j = e / a.out_dim;
    const int col = (int)(e - j * a.out_dim);
    const int c = col / sd;
    float v;
    if (c < a.n) v = in[(j * a.ns + a.first + a.ctx[c]) * a.dim + (col - c * sd)];
    else v = in[j * a.ns * a.dim + sd + (col - a.n * sd)];  // const part: the chunk's first row
    out[e] = v;
  }
}
// one thread per input element: a pure gather (no atomics): input row
// j * ns + s gets block c of output row j when first + ctx[c] == s
__global__ void k_splice_bwd(const float *__restrict__ od, long rows, SpliceArgs a, float *__restrict__ id) {
  const long total = rows * a.ns * a.dim;
  const int sd = a.dim - a.const_dim;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / a.dim;
    const int col = (int)(e - r * a.dim);
    const long j = r / a.ns;
    const int sp = (int)(r - j * a.ns);
    float v = 0.f;
    if (col < sd) {
      for (int c = 0; c < a.n; c++)
        if (a.first + a.ctx[c] == sp) v += od[j * a.out_dim + c * sd + col];
    } else if (sp == 0) {
      v = od[j * a.out_dim + a.n * sd + (col - sd)];
    }
    id[e] = v;
  }
}

static SpliceArgs splice_args(int dim, int ns, const int *ctx, int nctx, int first, int const_dim) {
  if (nctx <= 0 || nctx > kMaxSplice) throw std::invalid_argument("splice: 1..32 context offsets");
  SpliceArgs a{};
  a.n = nctx; a.first = first; a.dim = dim; a.const_dim = const_dim; a.ns = ns;
  a.out_dim = (dim - const_dim) * nctx + const_dim;
  for (int c = 0; c < nctx; c++) a.ctx[c] = ctx[c];
  return a;
}

void splice_rows(hipStream_t s, const float *in, int dim, int ns, long rows, const int *ctx, int nctx, int first,
                 int const_dim, float *out) {
  if (rows <= 0) return;
  const SpliceArgs a = splice_args(dim, ns, ctx, nctx, first, const_dim);
  hipLaunchKernelGGL(k_splice, dim3(grid_for(rows * a.out_dim)), dim3(256), 0, s, in, rows, a, out);
}

void splice_rows_backward(hipStream_t s, const float *out_deriv, int dim, int ns, long rows, const int *ctx, int nctx,
                          int first, int const_dim, float *in_deriv) {
  if (rows <= 0) return;
  const SpliceArgs a = splice_args(dim, ns, ctx, nctx, first, const_dim);
  hipLaunchKernelGGL(k_splice_bwd, dim3(grid_for(rows * ns * dim)), dim3(256), 0, s, out_deriv, rows, a, in_deriv);
}

__global__ void k_pad_splice(const float *__restrict__ feats, int T, int dim, int left, int ns,
                             float *__restrict__ out) {
  const long total = (long)T * ns * dim;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long r = e / dim;
    const int col = (int)(e - r * dim);
    const int t = (int)(r / ns), sp = (int)(r - (long)t * ns);
    const int src = min(max(t + sp - left, 0), T - 1);
    out[e] = feats[(long)src * dim + col];
  }
}

void pad_splice_input(hipStream_t s, const float *feats, int T, int dim, int left, int ns, float *out) {
  if (T <= 0 || dim <= 0 || ns <= 0) return;
  hipLaunchKernelGGL(k_pad_splice, dim3(grid_for((long)T * ns * dim)), dim3(256), 0, s, feats, T, dim, left, ns, out);
}

// ---- data-parallel step agreement ------------------------------------------
__global__ void k_err_to_flag(const unsigned *err, float *flag) { flag[0] = err[0] ? 1.f : 0.f; }
__global__ void k_flag_to_err(const float *flag, unsigned *err) {
  if (flag[0] > 0.f) err[0] |= kErrPeerFailed;
}

void err_word_to_flag(hipStream_t s, const unsigned *err, float *flag) {
  hipLaunchKernelGGL(k_err_to_flag, dim3(1), dim3(1), 0, s, err, flag);
}
void flag_to_err_word(hipStream_t s, const float *flag, unsigned *err) {
  hipLaunchKernelGGL(k_flag_to_err, dim3(1), dim3(1), 0, s, flag, err);
}

// ---- CU occupancy probe ----------------------------------------------------
// Every block takes a whole CU (1024 threads, the dynamic LDS below) and
// stays resident for `ticks` of the 100-MHz constant clock; every wave leaves
// on the same time test, so the grid always drains.
__global__ __launch_bounds__(1024) void k_cu_hold(unsigned long long ticks) {
  extern __shared__ float hold_lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) hold_lds[0] = 0.f;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

__global__ __launch_bounds__(64) void k_cu_where(unsigned *ids, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned x, h;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
  if (threadIdx.x == 0) ids[blockIdx.x] = ((x & 0xfu) << 16) | ((h >> 8) & 0xffu);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void cu_where(hipStream_t s, unsigned *ids, int blocks, double usec) {
  if (blocks <= 0) return;
  hipLaunchKernelGGL(k_cu_where, dim3(blocks), dim3(64), 0, s, ids, (unsigned long long)(usec * 100.0));
  KCTC_HIP_CHECK(hipGetLastError());
}

void cu_hold(hipStream_t s, int blocks, double usec) {
  if (blocks <= 0 || usec <= 0) return;
  const int lds = 160 * 1024;
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_cu_hold),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(k_cu_hold, dim3(blocks), dim3(1024), lds, s, (unsigned long long)(usec * 100.0));
  KCTC_HIP_CHECK(hipGetLastError());
}

}  // namespace kctc
