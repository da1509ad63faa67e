// rnn.hip -- cuDNN-v5 compatible LSTM / GRU / RELU / TANH layers for gfx950.
//
// Forward (per stacked layer):
//   1. G = x W^T + bW (+ bR for LSTM/RNN)      one batched fp32 MFMA GEMM for both
//      directions (gemm.hip): the input projection of all T*N frames at once.
//   2. rnn_fwd_rec<MODE>: ONE persistent launch runs the whole time recurrence of
//      both directions.  Workgroup (dir, g) owns hidden units [g*U, g*U+U): its
//      slice of R (nW*U rows x H, fp32) is loaded into LDS once, its cell
//      state stays in registers for all T steps.  Per step it multiplies
//      h_{t-1} [N x H] by the slice on the matrix cores (v_mfma_f32_16x16x4_f32,
//      K split over the 4 waves, reduced through LDS), applies the gate
//      nonlinearities and publishes its U columns of h_t.
//      Inter-workgroup hand-off: the layer output y (= the h exchange buffer)
//      is pre-filled with a NaN sentinel; h_t is published with write-through
//      (sc1) 4-byte stores and consumers read h_{t-1} straight into MFMA
//      A-operand registers with sc1 16-byte buffer loads, re-polling any
//      fragment that still holds the sentinel (data-as-flag: no barrier, no
//      flag word; each 4-byte store is a granule; MI355X_MICROARCH.md §R2).
//      Spins are bounded; a timeout sets a device error word and every
//      workgroup drains out.
// Backward data: rnn_bwd_rec<MODE>, the mirror image: workgroup (dir, g) owns
//   units [g*U, g*U+U) and keeps R^T's U rows (U x nW*H) in LDS; per step it
//   polls dGates_{t+1} (all nW*H columns) from a sentinel-filled exchange
//   buffer E, forms dh = dy + dGates_{t+1} R on the matrix cores, does the
//   pointwise cell backward (dc carried in registers) and publishes its
//   dGates_t columns.  E is kept in the reserve for backward-weights.
// Backward weights: dW += dGx^T x, dR += dGh^T h_prev (time-shifted views of E
//   and y; batched over directions), bias sums accumulated by the recurrence.
//
// Semantics follow cuDNN v5 as used by CuDNNRecurrentComponent: hx = cx = 0,
// dhy = dcy = 0 (SetBufferZero, nnet-cudnn-component.cc:494-506), all N
// sequences run the full T steps (no masking), weights in the opaque layout of
// nnet-cudnn-component.cc:327-413 (see RnnDesc::lin_offset).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "elementwise.h"
#include "gemm.h"
#include "prof.h"
#include "rnn.h"

namespace kctc {

long RnnDesc::params_size() const {
  long t = 0;
  for (int l = 0; l < layers; l++) t += dirs * pl_size(l);
  return t;
}

long RnnDesc::lin_offset(int p, int lin, bool bias) const {
  long off = 0;
  for (int q = 0; q < p; q++) off += pl_size(q / dirs);
  const int layer = p / dirs, di = din(layer);
  const long n = nw();
  if (!bias) {
    if (lin < n) return off + (long)lin * H * di;
    return off + n * H * (long)di + (long)(lin - n) * H * H;
  }
  return off + n * H * (long)di + n * H * (long)H + (long)lin * H;
}

static long al64(long x) { return (x + 63) / 64 * 64; }

RnnReserveLayout rnn_reserve_layout(const RnnDesc &d, int T, int N) {
  RnnReserveLayout r;
  const long TN = (long)T * N, nw = d.nw(), H = d.H, dirs = d.dirs;
  long p = 0;
  r.G = p;    p += al64(TN * dirs * nw * H);
  r.aux = p;  p += al64(TN * dirs * H);
  r.E = p;    p += al64(TN * dirs * nw * H);
  r.DX = p;   p += (d.mode == kGru) ? al64(TN * dirs * nw * H) : 0;
  r.bias = p; p += al64(dirs * 2 * nw * H);
  r.out = p;  p += (d.layers > 1) ? al64(TN * dirs * H) : 0;
  r.dout = p; p += (d.layers > 1) ? al64(TN * dirs * H) : 0;
  r.per_layer = p;
  r.total = p * d.layers;
  return r;
}

static long drec_split_floats(const RnnDesc &d, int T, int N) {
  long need = 0;
  const int G4 = d.nw() * d.H;
  for (int l = 0; l < d.layers; l++) {
    const long K = (long)(T > 1 ? T - 1 : 1) * N;
    int s = gemm_pick_split(G4, d.H, (int)K, d.dirs);
    if (s > 1) need = std::max(need, (long)s * d.dirs * G4 * d.H);
    s = gemm_pick_split(G4, d.din(l), (int)((long)T * N), d.dirs);
    if (s > 1) need = std::max(need, (long)s * d.dirs * G4 * d.din(l));
  }
  return need;
}

size_t rnn_workspace_bytes(const RnnDesc &d, int T, int N) {
  return sizeof(float) * (size_t)al64(drec_split_floats(d, T, N)) + 256;
}

namespace {

constexpr int NT = 256;
constexpr unsigned kSent = 0xFFFFFFFFu;
constexpr int kSpinLimit = 1 << 21;
constexpr int kCH = 8;   // k-groups (16 k each) of A fragments in flight per wave
constexpr int kMaxRT = 4;  // N <= 64 (four 16-row MFMA tiles)
constexpr int kMaxCT = 4;  // <= 64 gate columns per workgroup
constexpr int kMaxIPT = 4;  // pointwise items per thread (N*U <= 1024)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool ready4(u32x4 v) {
  return (v[0] != kSent) & (v[1] != kSent) & (v[2] != kSent) & (v[3] != kSent);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16 /* sc1 */);
}

// Re-poll one 16-byte fragment until it holds no sentinel (bounded spin).
__device__ __forceinline__ u32x4 settle(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v,
                                        unsigned *err, int &bad) {
  int spins = 0;
  while (!bad && !ready4(v)) {
    if (++spins > kSpinLimit) { bad = 1; break; }
    if ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      bad = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    v = ld_sc1(r, off);
  }
  return v;
}

__device__ __forceinline__ void publish(float *p, float v) {
  unsigned u = __float_as_uint(v);
  if (u == kSent) u = 0x7FC00000u;  // never publish the sentinel bit pattern
  __hip_atomic_store(reinterpret_cast<unsigned *>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

struct RecParams {
  int T, N, H, dirs, U, nwg, ncol, Npad;
  const float *w;   // params base of this stacked layer's pseudo-layer 0
  long pl_stride;   // floats between the two directions' blocks
  long r_off;       // R within a pseudo-layer block
  long bR_off;      // bR within a pseudo-layer block
  float *G;         // [T*N][dirs*nW*H] pre-activations -> activations
  float *y;         // [T*N][dirs*H] output / h exchange (sentinel pre-filled)
  float *aux;       // LSTM: c ; GRU: R_n h + b_Rn   [T*N][dirs*H]
  const float *dy;  // backward: [T*N][dirs*H]
  float *E;         // backward: dGates (recurrent part) exchange [T*N][dirs*nW*H]
  float *DX;        // backward GRU: dGates (input part); == E otherwise
  float *bias;      // backward: bias partial sums [dirs][2][nW*H]
  unsigned *err;
};

// ---------------------------------------------------------------------------
// forward recurrence
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(NT, 1) void rnn_fwd_rec(RecParams p) {
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int H = p.H, U = p.U, N = p.N, T = p.T, ncol = p.ncol;
  const int LDR = H + 4;
  const int d = blockIdx.x / p.nwg, u0 = (blockIdx.x % p.nwg) * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int RT = p.Npad / 16, CT = ncol / 16;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *Rs = smem;                      // [ncol][LDR]
  float *red = Rs + (long)ncol * LDR;    // [4][Npad][ncol]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  for (int idx = tid; idx < ncol * H; idx += NT) {
    const int c = idx / H, k = idx - c * H;
    float v = 0.f;
    if (c < NW * U) {
      const int gt = c / U, u = c - gt * U;
      v = R[(long)(gt * H + u0 + u) * H + k];
    }
    Rs[c * LDR + k] = v;
  }
  // pointwise items (n, u)
  const int items = N * U;
  float cst[kMaxIPT], hpv[kMaxIPT], gin[kMaxIPT][NW], bR[kMaxIPT][NW];
#pragma unroll
  for (int j = 0; j < kMaxIPT; j++) {
    cst[j] = 0.f;
    hpv[j] = 0.f;
    const int it = tid + j * NT, u = it % U;
#pragma unroll
    for (int g = 0; g < NW; g++) {
      bR[j][g] = (MODE == kGru && it < items) ? Wd[p.bR_off + g * H + u0 + u] : 0.f;
      gin[j][g] = 0.f;
    }
  }
  // prefetch the input projection of the first step
  {
    const int t = d == 0 ? 0 : T - 1;
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
#pragma unroll
        for (int g = 0; g < NW; g++)
          gin[j][g] = p.G[((long)t * N + n) * ldg + (long)d * NW * H + g * H + u0 + u];
      }
    }
  }
  __syncthreads();
  int bad = 0;
  const int KG = H / 16;  // k-groups, dealt round-robin to the 4 waves
  const unsigned step_bytes = (unsigned)((long)N * ldy * sizeof(float));
  for (int k = 0; k < T; k++) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    floatx4 acc[kMaxRT][kMaxCT];
#pragma unroll
    for (int a = 0; a < kMaxRT; a++)
#pragma unroll
      for (int b = 0; b < kMaxCT; b++) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (k > 0) {
      const auto rs = rsrc(p.y + (long)tp * N * ldy, step_bytes);
      for (int c0 = w; c0 < KG; c0 += 4 * kCH) {
        u32x4 af[kMaxRT][kCH];
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
#pragma unroll
          for (int rt = 0; rt < kMaxRT; rt++) {
            const int n = rt * 16 + fr;
            af[rt][i] = u32x4{0u, 0u, 0u, 0u};
            if (rt < RT && kg < KG && n < N)
              af[rt][i] = ld_sc1(rs, (unsigned)(((long)n * ldy + (long)d * H + kg * 16 + fq * 4) * 4));
          }
        }
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
#pragma unroll
          for (int rt = 0; rt < kMaxRT; rt++) {
            const int n = rt * 16 + fr;
            if (rt < RT && kg < KG && n < N)
              af[rt][i] = settle(rs, (unsigned)(((long)n * ldy + (long)d * H + kg * 16 + fq * 4) * 4),
                                 af[rt][i], p.err, bad);
          }
        }
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
          if (kg < KG) {
#pragma unroll
            for (int ct = 0; ct < kMaxCT; ct++) {
              if (ct < CT) {
                const floatx4 b = *reinterpret_cast<const floatx4 *>(Rs + (ct * 16 + fr) * LDR + kg * 16 + fq * 4);
#pragma unroll
                for (int s = 0; s < 4; s++)
#pragma unroll
                  for (int rt = 0; rt < kMaxRT; rt++)
                    if (rt < RT)
                      acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                          __uint_as_float(af[rt][i][s]), b[s], acc[rt][ct], 0, 0, 0);
              }
            }
          }
        }
      }
    }
    // cross-wave K reduction through LDS
#pragma unroll
    for (int rt = 0; rt < kMaxRT; rt++)
#pragma unroll
      for (int ct = 0; ct < kMaxCT; ct++)
        if (rt < RT && ct < CT)
#pragma unroll
          for (int r = 0; r < 4; r++)
            red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * ncol + ct * 16 + fr] = acc[rt][ct][r];
    __syncthreads();
    // pointwise cell update for owned (n, u)
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        float rh[NW];
#pragma unroll
        for (int g = 0; g < NW; g++) {
          const int c = g * U + u;
          rh[g] = ((red[((long)0 * p.Npad + n) * ncol + c] + red[((long)1 * p.Npad + n) * ncol + c]) +
                   red[((long)2 * p.Npad + n) * ncol + c]) + red[((long)3 * p.Npad + n) * ncol + c];
        }
        const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
        const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
        float h;
        if (MODE == kLstm) {
          const float ig = sigm(gin[j][0] + rh[0]);
          const float fg = sigm(gin[j][1] + rh[1]);
          const float gg = tanhf(gin[j][2] + rh[2]);
          const float og = sigm(gin[j][3] + rh[3]);
          const float cc = fg * cst[j] + ig * gg;
          cst[j] = cc;
          h = og * tanhf(cc);
          p.G[grow] = ig; p.G[grow + H] = fg; p.G[grow + 2 * H] = gg; p.G[grow + 3 * H] = og;
          p.aux[yrow] = cc;
        } else if (MODE == kGru) {
          const float r = sigm(gin[j][0] + rh[0] + bR[j][0]);
          const float z = sigm(gin[j][1] + rh[1] + bR[j][1]);
          const float rhn = rh[2] + bR[j][2];
          const float nn = tanhf(gin[j][2] + r * rhn);
          h = (1.f - z) * nn + z * hpv[j];
          hpv[j] = h;
          p.G[grow] = r; p.G[grow + H] = z; p.G[grow + 2 * H] = nn;
          p.aux[yrow] = rhn;
        } else {
          const float pre = gin[j][0] + rh[0];
          h = MODE == kRelu ? fmaxf(pre, 0.f) : tanhf(pre);
        }
        publish(p.y + yrow, h);
        // prefetch the next step's input projection
        if (k + 1 < T) {
          const int tn = d == 0 ? t + 1 : t - 1;
#pragma unroll
          for (int g = 0; g < NW; g++)
            gin[j][g] = p.G[((long)tn * N + n) * ldg + (long)d * NW * H + g * H + u0 + u];
        }
      }
    }
    __syncthreads();  // red[] is rewritten by the next step
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

// ---------------------------------------------------------------------------
// backward-data recurrence
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_rec(RecParams p) {
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int H = p.H, U = p.U, N = p.N, T = p.T;
  const int K = NW * H, LDK = K + 4;
  const int d = blockIdx.x / p.nwg, u0 = (blockIdx.x % p.nwg) * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int RT = p.Npad / 16;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *RT_s = smem;                       // [U][LDK]: RT_s[u][kk] = R[kk][u0+u]
  float *red = RT_s + (long)U * LDK;        // [4][Npad][16]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  for (int idx = tid; idx < U * K; idx += NT) {
    const int kk = idx / U, u = idx - kk * U;
    RT_s[u * LDK + kk] = R[(long)kk * H + u0 + u];
  }
  const int items = N * U;
  float carry[kMaxIPT];   // LSTM: dc carried to the previous step; GRU: dh*z direct term
  float bsx[kMaxIPT][NW], bsh[kMaxIPT][NW];
#pragma unroll
  for (int j = 0; j < kMaxIPT; j++) {
    carry[j] = 0.f;
#pragma unroll
    for (int g = 0; g < NW; g++) bsx[j][g] = bsh[j][g] = 0.f;
  }
  __syncthreads();
  int bad = 0;
  const int KG = K / 16;
  const unsigned step_bytes = (unsigned)((long)N * ldg * sizeof(float));
  for (int k = T - 1; k >= 0; k--) {
    const int t = d == 0 ? k : T - 1 - k;       // forward-order index k
    const int tn = d == 0 ? t + 1 : t - 1;      // processed just before (k+1)
    const int tp = d == 0 ? t - 1 : t + 1;      // forward predecessor (k-1)
    floatx4 acc[kMaxRT];
#pragma unroll
    for (int a = 0; a < kMaxRT; a++) acc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (k < T - 1) {
      const auto rs = rsrc(p.E + (long)tn * N * ldg, step_bytes);
      for (int c0 = w; c0 < KG; c0 += 4 * kCH) {
        u32x4 af[kMaxRT][kCH];
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
#pragma unroll
          for (int rt = 0; rt < kMaxRT; rt++) {
            const int n = rt * 16 + fr;
            af[rt][i] = u32x4{0u, 0u, 0u, 0u};
            if (rt < RT && kg < KG && n < N)
              af[rt][i] = ld_sc1(rs, (unsigned)(((long)n * ldg + (long)d * K + kg * 16 + fq * 4) * 4));
          }
        }
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
#pragma unroll
          for (int rt = 0; rt < kMaxRT; rt++) {
            const int n = rt * 16 + fr;
            if (rt < RT && kg < KG && n < N)
              af[rt][i] = settle(rs, (unsigned)(((long)n * ldg + (long)d * K + kg * 16 + fq * 4) * 4),
                                 af[rt][i], p.err, bad);
          }
        }
#pragma unroll
        for (int i = 0; i < kCH; i++) {
          const int kg = c0 + 4 * i;
          if (kg < KG) {
            floatx4 b = floatx4{0.f, 0.f, 0.f, 0.f};
            if (fr < U) b = *reinterpret_cast<const floatx4 *>(RT_s + fr * LDK + kg * 16 + fq * 4);
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
              for (int rt = 0; rt < kMaxRT; rt++)
                if (rt < RT)
                  acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][i][s]), b[s],
                                                                 acc[rt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < kMaxRT; rt++)
      if (rt < RT)
#pragma unroll
        for (int r = 0; r < 4; r++) red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * 16 + fr] = acc[rt][r];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        const float dhr = ((red[((long)0 * p.Npad + n) * 16 + u] + red[((long)1 * p.Npad + n) * 16 + u]) +
                           red[((long)2 * p.Npad + n) * 16 + u]) + red[((long)3 * p.Npad + n) * 16 + u];
        const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
        const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
        float dh = p.dy[yrow] + dhr;
        if (MODE == kLstm) {
          const float ig = p.G[grow], fg = p.G[grow + H], gg = p.G[grow + 2 * H], og = p.G[grow + 3 * H];
          const float cc = p.aux[yrow];
          const float cp = k > 0 ? p.aux[((long)tp * N + n) * ldy + (long)d * H + u0 + u] : 0.f;
          const float tc = tanhf(cc);
          const float dO = dh * tc;
          const float dc = dh * og * (1.f - tc * tc) + carry[j];
          const float dpi = dc * gg * ig * (1.f - ig);
          const float dpf = dc * cp * fg * (1.f - fg);
          const float dpg = dc * ig * (1.f - gg * gg);
          const float dpo = dO * og * (1.f - og);
          carry[j] = dc * fg;
          publish(p.E + grow, dpi);
          publish(p.E + grow + H, dpf);
          publish(p.E + grow + 2 * H, dpg);
          publish(p.E + grow + 3 * H, dpo);
          bsx[j][0] += dpi; bsx[j][1] += dpf; bsx[j][2] += dpg; bsx[j][3] += dpo;
        } else if (MODE == kGru) {
          dh += carry[j];
          const float r = p.G[grow], z = p.G[grow + H], nn = p.G[grow + 2 * H];
          const float rhn = p.aux[yrow];
          const float hp = k > 0 ? p.y[((long)tp * N + n) * ldy + (long)d * H + u0 + u] : 0.f;
          const float dn = dh * (1.f - z), dz = dh * (hp - nn);
          const float dpn = dn * (1.f - nn * nn);
          const float dpr = dpn * rhn * r * (1.f - r);
          const float dpz = dz * z * (1.f - z);
          carry[j] = dh * z;
          p.DX[grow] = dpr; p.DX[grow + H] = dpz; p.DX[grow + 2 * H] = dpn;
          publish(p.E + grow, dpr);
          publish(p.E + grow + H, dpz);
          publish(p.E + grow + 2 * H, dpn * r);
          bsx[j][0] += dpr; bsx[j][1] += dpz; bsx[j][2] += dpn;
          bsh[j][0] += dpr; bsh[j][1] += dpz; bsh[j][2] += dpn * r;
        } else {
          const float h = p.y[yrow];
          const float der = MODE == kRelu ? (h > 0.f ? 1.f : 0.f) : (1.f - h * h);
          const float dp = dh * der;
          publish(p.E + grow, dp);
          bsx[j][0] += dp;
        }
      }
    }
    __syncthreads();
  }
  // bias partial sums: reduce over n in a fixed order through LDS
  float *bs = red;  // reuse: [items][NW] for x and h parts (needs <= 2*1024*4 floats)
#pragma unroll
  for (int j = 0; j < kMaxIPT; j++) {
    const int it = tid + j * NT;
    if (it < items)
#pragma unroll
      for (int g = 0; g < NW; g++) {
        bs[(long)it * NW + g] = bsx[j][g];
        bs[(long)items * NW + (long)it * NW + g] = (MODE == kGru) ? bsh[j][g] : bsx[j][g];
      }
  }
  __syncthreads();
  for (int q = tid; q < 2 * NW * U; q += NT) {
    const int part = q / (NW * U), rem = q - part * NW * U, g = rem / U, u = rem - g * U;
    float s = 0.f;
    for (int n = 0; n < N; n++) s += bs[(long)part * items * NW + ((long)n * U + u) * NW + g];
    p.bias[((long)d * 2 + part) * NW * H + g * H + u0 + u] = s;
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

template <typename F>
static void set_lds(F f, size_t bytes) {
  static size_t done[8] = {0};
  (void)done;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)bytes);
}

static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return v ? atoi(v) : dflt;
}

// pick U (units per workgroup): divides H, multiple of 4, blocks <= 256
static int pick_fwd_u(const RnnDesc &d, int N) {
  int want = env_int("KCTC_FWD_U", 0);
  const int NW = d.nw();
  auto ok = [&](int U) {
    if (U <= 0 || d.H % U || NW * U > 16 * kMaxCT || N * U > NT * kMaxIPT) return false;
    if ((long)d.dirs * (d.H / U) > 256) return false;
    const int ncol = (NW * U + 15) / 16 * 16, Npad = (N + 15) / 16 * 16;
    const size_t lds = sizeof(float) * ((size_t)ncol * (d.H + 4) + 4 * (size_t)Npad * ncol);
    return lds <= 160 * 1024;
  };
  if (want && ok(want)) return want;
  for (int U : {8, 4, 16, 2, 1})
    if (ok(U) && (long)d.dirs * (d.H / U) <= 128) return U;
  for (int U : {4, 8, 16, 2, 1})
    if (ok(U)) return U;
  return 0;
}

static int pick_bwd_u(const RnnDesc &d, int N) {
  int want = env_int("KCTC_BWD_U", 0);
  const int K = d.nw() * d.H;
  auto ok = [&](int U) {
    if (U <= 0 || U > 16 || d.H % U || N * U > NT * kMaxIPT) return false;
    if ((long)d.dirs * (d.H / U) > 256) return false;
    const int Npad = (N + 15) / 16 * 16;
    const size_t lds = sizeof(float) * ((size_t)U * (K + 4) + std::max(4 * (size_t)Npad * 16,
                                                                        (size_t)2 * N * U * d.nw()));
    return lds <= 160 * 1024;
  };
  if (want && ok(want)) return want;
  for (int U : {16, 8, 4, 2, 1})
    if (ok(U)) return U;
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// host: forward training
// ---------------------------------------------------------------------------
int rnn_forward_training(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *w, float *y, void *workspace, size_t ws_bytes,
                         void *reserve, size_t res_bytes, unsigned *err) {
  if (T <= 0 || N <= 0 || N > 16 * kMaxRT || d.H % 16) return KRNN_NOT_SUPPORTED;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
  const int U = pick_fwd_u(d, N);
  if (!U) return KRNN_NOT_SUPPORTED;
  const int NW = d.nw(), H = d.H, dirs = d.dirs;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  const float *in = x;
  for (int l = 0; l < d.layers; l++) {
    float *R0 = res + lay.per_layer * l;
    float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const float *wl = w + pl0;
    const long pls = d.pl_size(l);
    const long bW = d.lin_offset(l * dirs, 0, true) - pl0;
    const long bR = d.lin_offset(l * dirs, NW, true) - pl0;
    const long roff = d.lin_offset(l * dirs, NW, false) - pl0;
    KCTC_HIP_CHECK(hipMemsetAsync(out, 0xFF, sizeof(float) * TN * dirs * H, s));
    GemmArgs g;
    g.transA = false; g.transB = true;
    g.M = (int)TN; g.N = NW * H; g.K = Din;
    g.A = in; g.lda = Din;
    g.B = wl; g.ldb = Din;
    g.C = R0 + lay.G; g.ldc = (long)dirs * NW * H;
    g.bias = wl + bW;
    g.bias2 = (d.mode == kGru) ? nullptr : wl + bR;
    g.batch = dirs; g.strideA = 0; g.strideB = pls; g.strideC = (long)NW * H; g.strideBias = pls;
    {
      ProfSpan ps(s, "gemm_fwd_proj");
      gemm_f32(s, g);
    }
    RecParams p{};
    p.T = T; p.N = N; p.H = H; p.dirs = dirs; p.U = U; p.nwg = H / U;
    p.ncol = (NW * U + 15) / 16 * 16; p.Npad = (N + 15) / 16 * 16;
    p.w = wl; p.pl_stride = pls; p.r_off = roff; p.bR_off = bR;
    p.G = R0 + lay.G; p.y = out; p.aux = R0 + lay.aux; p.err = err;
    const size_t lds = sizeof(float) * ((size_t)p.ncol * (H + 4) + 4 * (size_t)p.Npad * p.ncol);
    const dim3 grid(dirs * p.nwg);
    ProfSpan ps(s, "rnn_fwd_rec");
    switch (d.mode) {
      case kLstm: set_lds(rnn_fwd_rec<kLstm>, lds);
        hipLaunchKernelGGL(rnn_fwd_rec<kLstm>, grid, dim3(NT), lds, s, p); break;
      case kGru: set_lds(rnn_fwd_rec<kGru>, lds);
        hipLaunchKernelGGL(rnn_fwd_rec<kGru>, grid, dim3(NT), lds, s, p); break;
      case kRelu: set_lds(rnn_fwd_rec<kRelu>, lds);
        hipLaunchKernelGGL(rnn_fwd_rec<kRelu>, grid, dim3(NT), lds, s, p); break;
      default: set_lds(rnn_fwd_rec<kTanh>, lds);
        hipLaunchKernelGGL(rnn_fwd_rec<kTanh>, grid, dim3(NT), lds, s, p); break;
    }
    KCTC_HIP_CHECK(hipGetLastError());
    in = out;
  }
  return KRNN_OK;
}

// ---------------------------------------------------------------------------
// host: backward data (dGates into the reserve, dx)
// ---------------------------------------------------------------------------
int rnn_backward_data(const RnnDesc &d, hipStream_t s, int T, int N, const float *y,
                      const float *dy, const float *w, float *dx, void *workspace,
                      size_t ws_bytes, void *reserve, size_t res_bytes, unsigned *err) {
  if (T <= 0 || N <= 0 || N > 16 * kMaxRT || d.H % 16) return KRNN_NOT_SUPPORTED;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  const int U = pick_bwd_u(d, N);
  if (!U) return KRNN_NOT_SUPPORTED;
  const int NW = d.nw(), H = d.H, dirs = d.dirs;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  const float *dcur = dy;
  for (int l = d.layers - 1; l >= 0; l--) {
    float *R0 = res + lay.per_layer * l;
    const float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const float *wl = w + pl0;
    const long pls = d.pl_size(l);
    float *E = R0 + lay.E;
    float *DX = d.mode == kGru ? R0 + lay.DX : E;
    KCTC_HIP_CHECK(hipMemsetAsync(E, 0xFF, sizeof(float) * TN * dirs * NW * H, s));
    RecParams p{};
    p.T = T; p.N = N; p.H = H; p.dirs = dirs; p.U = U; p.nwg = H / U;
    p.ncol = 16; p.Npad = (N + 15) / 16 * 16;
    p.w = wl; p.pl_stride = pls; p.r_off = d.lin_offset(l * dirs, NW, false) - pl0;
    p.bR_off = d.lin_offset(l * dirs, NW, true) - pl0;
    p.G = R0 + lay.G; p.y = const_cast<float *>(out); p.aux = R0 + lay.aux;
    p.dy = dcur; p.E = E; p.DX = DX; p.bias = R0 + lay.bias; p.err = err;
    const size_t lds = sizeof(float) * ((size_t)U * (NW * H + 4) +
                                        std::max(4 * (size_t)p.Npad * 16, (size_t)2 * N * U * NW));
    const dim3 grid(dirs * p.nwg);
    {
    ProfSpan ps(s, "rnn_bwd_rec");
    switch (d.mode) {
      case kLstm: set_lds(rnn_bwd_rec<kLstm>, lds);
        hipLaunchKernelGGL(rnn_bwd_rec<kLstm>, grid, dim3(NT), lds, s, p); break;
      case kGru: set_lds(rnn_bwd_rec<kGru>, lds);
        hipLaunchKernelGGL(rnn_bwd_rec<kGru>, grid, dim3(NT), lds, s, p); break;
      case kRelu: set_lds(rnn_bwd_rec<kRelu>, lds);
        hipLaunchKernelGGL(rnn_bwd_rec<kRelu>, grid, dim3(NT), lds, s, p); break;
      default: set_lds(rnn_bwd_rec<kTanh>, lds);
        hipLaunchKernelGGL(rnn_bwd_rec<kTanh>, grid, dim3(NT), lds, s, p); break;
    }
    }
    KCTC_HIP_CHECK(hipGetLastError());
    // dx_l = sum_dir DX_dir W_dir   (lower layer's dy, or the caller's dx)
    float *dxl = (l == 0) ? dx : res + lay.per_layer * (l - 1) + lay.dout;
    if (dxl) {
      for (int dir = 0; dir < dirs; dir++) {
        GemmArgs g;
        g.transA = false; g.transB = false;
        g.M = (int)TN; g.N = Din; g.K = NW * H;
        g.A = DX + (long)dir * NW * H; g.lda = (long)dirs * NW * H;
        g.B = wl + dir * pls; g.ldb = Din;
        g.C = dxl; g.ldc = Din;
        g.beta = dir == 0 ? 0.f : 1.f;
        ProfSpan ps(s, "gemm_bwd_data");
        gemm_f32(s, g);
      }
    }
    dcur = dxl;
  }
  return KRNN_OK;
}

// ---------------------------------------------------------------------------
// host: backward weights (accumulates into dw, like cudnnRNNBackwardWeights)
// ---------------------------------------------------------------------------
int rnn_backward_weights(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *y, void *workspace, size_t ws_bytes, float *dw,
                         void *reserve, size_t res_bytes) {
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
  const int NW = d.nw(), H = d.H, dirs = d.dirs, G4 = NW * H;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  float *ws = static_cast<float *>(workspace);
  for (int l = 0; l < d.layers; l++) {
    float *R0 = res + lay.per_layer * l;
    const float *in = l == 0 ? x : res + lay.per_layer * (l - 1) + lay.out;
    const float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const long pls = d.pl_size(l);
    float *dwl = dw + pl0;
    float *E = R0 + lay.E;
    float *DX = d.mode == kGru ? R0 + lay.DX : E;
    const long ldg = (long)dirs * G4, ldy = (long)dirs * H;
    // dW_dir += DX_dir^T x
    GemmArgs g;
    g.transA = true; g.transB = false;
    g.M = G4; g.N = Din; g.K = (int)TN;
    g.A = DX; g.lda = ldg; g.B = in; g.ldb = Din;
    g.C = dwl; g.ldc = Din; g.beta = 1.f;
    g.batch = dirs; g.strideA = G4; g.strideB = 0; g.strideC = pls;
    g.split_k = gemm_pick_split(g.M, g.N, g.K, dirs);
    g.ws = ws;
    {
      ProfSpan ps(s, "gemm_bwd_w");
      gemm_f32(s, g);
    }
    // dR_dir += E_dir(shifted)^T h_prev:  fwd pairs rows t>=1 with y rows t-1,
    // bwd pairs rows t<=T-2 with y rows t+1 (column half H..2H-1)
    if (T > 1) {
      GemmArgs r;
      r.transA = true; r.transB = false;
      r.M = G4; r.N = H; r.K = (int)((long)(T - 1) * N);
      r.A = E + (long)N * ldg; r.lda = ldg;
      r.B = out; r.ldb = ldy;
      r.C = dwl + (d.lin_offset(l * dirs, NW, false) - pl0); r.ldc = H; r.beta = 1.f;
      r.batch = dirs;
      r.strideA = (long)G4 - (long)N * ldg;        // dir 1: E + G4 (rows 0..T-2)
      r.strideB = (long)N * ldy + H;               // dir 1: y rows 1..T-1, cols H..
      r.strideC = pls;
      r.split_k = gemm_pick_split(r.M, r.N, r.K, dirs);
      r.ws = ws;
      ProfSpan ps(s, "gemm_bwd_r");
      gemm_f32(s, r);
    }
    // biases: dbW += sum dGx, dbR += sum dGh (partials from the recurrence)
    const long bW = d.lin_offset(l * dirs, 0, true) - pl0;
    const long bR = d.lin_offset(l * dirs, NW, true) - pl0;
    for (int dir = 0; dir < dirs; dir++) {
      const float *part = R0 + lay.bias + (long)dir * 2 * G4;
      clip_sgd_update(s, dwl + dir * pls + bW, part, G4, 1.f, 0.f);
      clip_sgd_update(s, dwl + dir * pls + bR, part + G4, G4, 1.f, 0.f);
    }
  }
  return KRNN_OK;
}

}  // namespace kctc
