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

// split-K slabs of the weight-gradient GEMMs, then the recurrence flag words
static size_t flags_offset(const RnnDesc &d, int T, int N) {
  return sizeof(float) * (size_t)al64(drec_split_floats(d, T, N));
}
size_t rnn_workspace_bytes(const RnnDesc &d, int T, int N) { return flags_offset(d, T, N) + 4096; }

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
  unsigned *flags;  // flag protocol: [dirs][nwg] step epochs, zeroed before launch
  unsigned *err;
  int sync;         // kSyncData / kSyncFlag
};

// Hand-off protocols (selected per launch; both placement-independent):
//  kSyncData: the payload is the flag (sentinel-filled buffer, sc1 4-B stores,
//             sc1 16-B loads re-polled until no sentinel is left).
//  kSyncFlag: payload sc1 stores -> every storing wave s_waitcnt vmcnt(0) ->
//             workgroup barrier -> ONE lane stores the step epoch (sc1) into
//             the workgroup's flag word; consumers: wave 0 polls the nwg flag
//             words of its direction with one sc1 load per lane, barrier, then
//             every wave loads the payload with sc1 loads (MI355X_MICROARCH.md
//             "Valid forms", row 1).  Polling traffic: 4 B per producer, not
//             the whole payload.
enum { kSyncData = 0, kSyncFlag = 1 };

__device__ __forceinline__ void wait_flags(const unsigned *flags, int nwg, unsigned epoch,
                                           unsigned *err, int &bad, int *bad_lds) {
  if (threadIdx.x < 64) {
    int spins = 0;
    while (true) {
      bool ok = true;
      for (int i = threadIdx.x; i < nwg; i += 64)
        ok &= __hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      if (++spins > kSpinLimit ||
          ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        bad = 1;
        if (threadIdx.x == 0) *bad_lds = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (*bad_lds) bad = 1;
}

__device__ __forceinline__ void signal_flag(unsigned *flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A-operand fragments of one step: rows n (RT 16-row tiles) x this wave's
// k-groups {w, w+4, ...}, CH k-groups per pass, straight from the exchange
// buffer into registers with sc1 16-B loads.  Returns false on timeout.
template <int RT, int CH>
__device__ __forceinline__ void load_frags(u32x4 (&af)[RT][CH], __amdgpu_buffer_rsrc_t rs, long ld,
                                           long col0, int c0, int KG, int N, int sync, unsigned *err,
                                           int &bad) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < CH; i++) {
    const int kg = w + 4 * (c0 + i);
#pragma unroll
    for (int rt = 0; rt < RT; rt++) {
      const int n = rt * 16 + fr;
      af[rt][i] = u32x4{0u, 0u, 0u, 0u};
      if (kg < KG && n < N) af[rt][i] = ld_sc1(rs, (unsigned)(((long)n * ld + col0 + kg * 16 + fq * 4) * 4));
    }
  }
  if (sync == kSyncData) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int kg = w + 4 * (c0 + i);
#pragma unroll
      for (int rt = 0; rt < RT; rt++) {
        const int n = rt * 16 + fr;
        if (kg < KG && n < N)
          af[rt][i] = settle(rs, (unsigned)(((long)n * ld + col0 + kg * 16 + fq * 4) * 4), af[rt][i], err, bad);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward recurrence
// ---------------------------------------------------------------------------
template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_fwd_rec(RecParams p) {
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  constexpr int CH = 32 / RT;  // k-groups per wave per pass (<= 32 A-fragment registers x4)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds;
  const int H = p.H, U = p.U, N = p.N, T = p.T, ncol = p.ncol;
  const int LDR = H + 4;
  const int d = blockIdx.x / p.nwg, g = blockIdx.x % p.nwg, u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int CT = ncol / 16;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *Rs = smem;                      // [ncol][LDR]
  float *red = Rs + (long)ncol * LDR;    // [4][Npad][ncol]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
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
    for (int q = 0; q < NW; q++) {
      bR[j][q] = (MODE == kGru && it < items) ? Wd[p.bR_off + q * H + u0 + u] : 0.f;
      gin[j][q] = 0.f;
    }
  }
  {  // prefetch the input projection of the first step
    const int t = d == 0 ? 0 : T - 1;
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
#pragma unroll
        for (int q = 0; q < NW; q++)
          gin[j][q] = p.G[((long)t * N + n) * ldg + (long)d * NW * H + q * H + u0 + u];
      }
    }
  }
  __syncthreads();
  int bad = 0;
  const int KG = H / 16;
  const int KGW = (KG + 3) / 4;  // k-groups per wave
  const unsigned step_bytes = (unsigned)((long)N * ldy * sizeof(float));
  unsigned *myflag = p.flags + d * p.nwg + g;
  for (int k = 0; k < T; k++) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    floatx4 acc[RT][kMaxCT];
#pragma unroll
    for (int a = 0; a < RT; a++)
#pragma unroll
      for (int b = 0; b < kMaxCT; b++) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (k > 0) {
      if (p.sync == kSyncFlag) wait_flags(p.flags + d * p.nwg, p.nwg, (unsigned)k, p.err, bad, &bad_lds);
      const auto rs = rsrc(p.y + (long)tp * N * ldy, step_bytes);
      for (int c0 = 0; c0 < KGW; c0 += CH) {
        u32x4 af[RT][CH];
        load_frags<RT, CH>(af, rs, ldy, (long)d * H, c0, KG, N, p.sync, p.err, bad);
#pragma unroll
        for (int i = 0; i < CH; i++) {
          const int kg = w + 4 * (c0 + i);
          if (kg < KG) {
#pragma unroll
            for (int ct = 0; ct < kMaxCT; ct++) {
              if (ct < CT) {
                const floatx4 b = *reinterpret_cast<const floatx4 *>(Rs + (ct * 16 + fr) * LDR + kg * 16 + fq * 4);
#pragma unroll
                for (int s = 0; s < 4; s++)
#pragma unroll
                  for (int rt = 0; rt < RT; rt++)
                    acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][i][s]), b[s],
                                                                       acc[rt][ct], 0, 0, 0);
              }
            }
          }
        }
      }
    }
    // cross-wave K reduction through LDS
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int ct = 0; ct < kMaxCT; ct++)
        if (ct < CT)
#pragma unroll
          for (int r = 0; r < 4; r++)
            red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * ncol + ct * 16 + fr] = acc[rt][ct][r];
    __syncthreads();
    // pointwise cell update for owned (n, u); publish h_t first, then the rest
    float act[kMaxIPT][NW], cnew[kMaxIPT];
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        float rh[NW];
#pragma unroll
        for (int q = 0; q < NW; q++) {
          const int c = q * U + u;
          rh[q] = ((red[((long)0 * p.Npad + n) * ncol + c] + red[((long)1 * p.Npad + n) * ncol + c]) +
                   red[((long)2 * p.Npad + n) * ncol + c]) + red[((long)3 * p.Npad + n) * ncol + c];
        }
        const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
        float h;
        if (MODE == kLstm) {
          act[j][0] = sigm(gin[j][0] + rh[0]);
          act[j][1] = sigm(gin[j][1] + rh[1]);
          act[j][2] = tanhf(gin[j][2] + rh[2]);
          act[j][3] = sigm(gin[j][3] + rh[3]);
          const float cc = act[j][1] * cst[j] + act[j][0] * act[j][2];
          cst[j] = cc;
          cnew[j] = cc;
          h = act[j][3] * tanhf(cc);
        } else if (MODE == kGru) {
          act[j][0] = sigm(gin[j][0] + rh[0] + bR[j][0]);
          act[j][1] = sigm(gin[j][1] + rh[1] + bR[j][1]);
          cnew[j] = rh[2] + bR[j][2];
          act[j][2] = tanhf(gin[j][2] + act[j][0] * cnew[j]);
          h = (1.f - act[j][1]) * act[j][2] + act[j][1] * hpv[j];
          hpv[j] = h;
        } else {
          const float pre = gin[j][0] + rh[0];
          h = MODE == kRelu ? fmaxf(pre, 0.f) : tanhf(pre);
        }
        publish(p.y + yrow, h);
      }
    }
    if (p.sync == kSyncFlag) signal_flag(myflag, (unsigned)(k + 1));
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
        const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
        if (MODE != kRelu && MODE != kTanh) {
#pragma unroll
          for (int q = 0; q < NW; q++) p.G[grow + q * H] = act[j][q];
          p.aux[yrow] = cnew[j];
        }
        if (k + 1 < T) {  // prefetch the next step's input projection
          const int tn = d == 0 ? t + 1 : t - 1;
#pragma unroll
          for (int q = 0; q < NW; q++)
            gin[j][q] = p.G[((long)tn * N + n) * ldg + (long)d * NW * H + q * H + u0 + u];
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
template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_rec(RecParams p) {
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  constexpr int CH = 32 / RT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds;
  const int H = p.H, U = p.U, N = p.N, T = p.T;
  const int K = NW * H, LDK = K + 4;
  const int d = blockIdx.x / p.nwg, g = blockIdx.x % p.nwg, u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *RT_s = smem;                       // [U][LDK]: RT_s[u][kk] = R[kk][u0+u]
  float *red = RT_s + (long)U * LDK;        // [4][Npad][16]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int idx = tid; idx < U * K; idx += NT) {
    const int kk = idx / U, u = idx - kk * U;
    RT_s[u * LDK + kk] = R[(long)kk * H + u0 + u];
  }
  const int items = N * U;
  float carry[kMaxIPT];   // LSTM: dc carried to the previous step; GRU: dh*z direct term
  float bsx[kMaxIPT][NW], bsh[kMaxIPT][NW];
  // prefetched pointwise operands of the step about to be processed
  float pdy[kMaxIPT], pg[kMaxIPT][NW], pa[kMaxIPT], pap[kMaxIPT];
#pragma unroll
  for (int j = 0; j < kMaxIPT; j++) {
    carry[j] = 0.f;
#pragma unroll
    for (int q = 0; q < NW; q++) bsx[j][q] = bsh[j][q] = pg[j][q] = 0.f;
    pdy[j] = pa[j] = pap[j] = 0.f;
  }
  auto prefetch = [&](int k) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
        const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
        const long prow = ((long)tp * N + n) * ldy + (long)d * H + u0 + u;
        pdy[j] = p.dy[yrow];
        if (MODE == kLstm || MODE == kGru) {
#pragma unroll
          for (int q = 0; q < NW; q++) pg[j][q] = p.G[grow + q * H];
          pa[j] = p.aux[yrow];
        }
        if (MODE == kLstm) pap[j] = k > 0 ? p.aux[prow] : 0.f;
        else if (MODE == kGru) pap[j] = k > 0 ? p.y[prow] : 0.f;
        else pap[j] = p.y[yrow];
      }
    }
  };
  prefetch(T - 1);
  __syncthreads();
  int bad = 0;
  const int KG = K / 16;
  const int KGW = (KG + 3) / 4;
  const unsigned step_bytes = (unsigned)((long)N * ldg * sizeof(float));
  unsigned *myflag = p.flags + d * p.nwg + g;
  for (int k = T - 1; k >= 0; k--) {
    const int t = d == 0 ? k : T - 1 - k;       // forward-order index k
    const int tn = d == 0 ? t + 1 : t - 1;      // processed just before (k+1)
    const unsigned epoch = (unsigned)(T - k);   // number of steps published so far
    floatx4 acc[RT];
#pragma unroll
    for (int a = 0; a < RT; a++) acc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (k < T - 1) {
      if (p.sync == kSyncFlag) wait_flags(p.flags + d * p.nwg, p.nwg, epoch - 1, p.err, bad, &bad_lds);
      const auto rs = rsrc(p.E + (long)tn * N * ldg, step_bytes);
      for (int c0 = 0; c0 < KGW; c0 += CH) {
        u32x4 af[RT][CH];
        load_frags<RT, CH>(af, rs, ldg, (long)d * K, c0, KG, N, p.sync, p.err, bad);
#pragma unroll
        for (int i = 0; i < CH; i++) {
          const int kg = w + 4 * (c0 + i);
          if (kg < KG) {
            floatx4 b = floatx4{0.f, 0.f, 0.f, 0.f};
            if (fr < U) b = *reinterpret_cast<const floatx4 *>(RT_s + fr * LDK + kg * 16 + fq * 4);
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
              for (int rt = 0; rt < RT; rt++)
                acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][i][s]), b[s], acc[rt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int r = 0; r < 4; r++) red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * 16 + fr] = acc[rt][r];
    __syncthreads();
    float dx_keep[kMaxIPT][NW];
#pragma unroll
    for (int j = 0; j < kMaxIPT; j++) {
      const int it = tid + j * NT;
      if (it < items) {
        const int n = it / U, u = it - n * U;
        const float dhr = ((red[((long)0 * p.Npad + n) * 16 + u] + red[((long)1 * p.Npad + n) * 16 + u]) +
                           red[((long)2 * p.Npad + n) * 16 + u]) + red[((long)3 * p.Npad + n) * 16 + u];
        const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
        float dh = pdy[j] + dhr;
        if (MODE == kLstm) {
          const float ig = pg[j][0], fg = pg[j][1], gg = pg[j][2], og = pg[j][3];
          const float cc = pa[j], cp = pap[j];
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
          const float r = pg[j][0], z = pg[j][1], nn = pg[j][2];
          const float rhn = pa[j], hp = pap[j];
          const float dn = dh * (1.f - z), dz = dh * (hp - nn);
          const float dpn = dn * (1.f - nn * nn);
          const float dpr = dpn * rhn * r * (1.f - r);
          const float dpz = dz * z * (1.f - z);
          carry[j] = dh * z;
          dx_keep[j][0] = dpr; dx_keep[j][1] = dpz; dx_keep[j][2] = dpn;
          publish(p.E + grow, dpr);
          publish(p.E + grow + H, dpz);
          publish(p.E + grow + 2 * H, dpn * r);
          bsx[j][0] += dpr; bsx[j][1] += dpz; bsx[j][2] += dpn;
          bsh[j][0] += dpr; bsh[j][1] += dpz; bsh[j][2] += dpn * r;
        } else {
          const float h = pap[j];
          const float der = MODE == kRelu ? (h > 0.f ? 1.f : 0.f) : (1.f - h * h);
          const float dp = dh * der;
          publish(p.E + grow, dp);
          bsx[j][0] += dp;
        }
      }
    }
    if (p.sync == kSyncFlag) signal_flag(myflag, epoch);
    if (MODE == kGru) {
#pragma unroll
      for (int j = 0; j < kMaxIPT; j++) {
        const int it = tid + j * NT;
        if (it < items) {
          const int n = it / U, u = it - n * U;
          const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
          p.DX[grow] = dx_keep[j][0]; p.DX[grow + H] = dx_keep[j][1]; p.DX[grow + 2 * H] = dx_keep[j][2];
        }
      }
    }
    if (k > 0) prefetch(k - 1);
    __syncthreads();
  }
  // bias partial sums: reduce over n in a fixed order through LDS
  float *bs = red;  // reuse: [items][NW] for x and h parts (needs <= 2*1024*4 floats)
#pragma unroll
  for (int j = 0; j < kMaxIPT; j++) {
    const int it = tid + j * NT;
    if (it < items)
#pragma unroll
      for (int q = 0; q < NW; q++) {
        bs[(long)it * NW + q] = bsx[j][q];
        bs[(long)items * NW + (long)it * NW + q] = (MODE == kGru) ? bsh[j][q] : bsx[j][q];
      }
  }
  __syncthreads();
  for (int q = tid; q < 2 * NW * U; q += NT) {
    const int part = q / (NW * U), rem = q - part * NW * U, gt = rem / U, u = rem - gt * U;
    float s = 0.f;
    for (int n = 0; n < N; n++) s += bs[(long)part * items * NW + ((long)n * U + u) * NW + gt];
    p.bias[((long)d * 2 + part) * NW * H + gt * H + u0 + u] = s;
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

template <int MODE, int RT>
static void launch_one(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  if (fwd) {
    set_lds(rnn_fwd_rec<MODE, RT>, lds);
    hipLaunchKernelGGL((rnn_fwd_rec<MODE, RT>), grid, dim3(NT), lds, s, p);
  } else {
    set_lds(rnn_bwd_rec<MODE, RT>, lds);
    hipLaunchKernelGGL((rnn_bwd_rec<MODE, RT>), grid, dim3(NT), lds, s, p);
  }
}
template <int MODE>
static void launch_mode(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  switch (p.Npad / 16) {
    case 1: launch_one<MODE, 1>(fwd, p, grid, lds, s); break;
    case 2: launch_one<MODE, 2>(fwd, p, grid, lds, s); break;
    case 3: launch_one<MODE, 3>(fwd, p, grid, lds, s); break;
    default: launch_one<MODE, 4>(fwd, p, grid, lds, s); break;
  }
}
static void launch_rec(bool fwd, int mode, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  switch (mode) {
    case kLstm: launch_mode<kLstm>(fwd, p, grid, lds, s); break;
    case kGru: launch_mode<kGru>(fwd, p, grid, lds, s); break;
    case kRelu: launch_mode<kRelu>(fwd, p, grid, lds, s); break;
    default: launch_mode<kTanh>(fwd, p, grid, lds, s); break;
  }
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
  // smallest U that keeps every workgroup resident (<= 256 = one per CU):
  // per-step MFMA latency falls with U (measured: U=4 < 8 < 16 on BLSTM-512)
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
    p.sync = env_int("KCTC_SYNC", kSyncFlag);
    p.flags = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
    KCTC_HIP_CHECK(hipMemsetAsync(p.flags, 0, 4096, s));
    const size_t lds = sizeof(float) * ((size_t)p.ncol * (H + 4) + 4 * (size_t)p.Npad * p.ncol);
    const dim3 grid(dirs * p.nwg);
    ProfSpan ps(s, "rnn_fwd_rec");
    launch_rec(true, d.mode, p, grid, lds, s);
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
    p.sync = env_int("KCTC_SYNC", kSyncFlag);
    if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
    p.flags = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
    KCTC_HIP_CHECK(hipMemsetAsync(p.flags, 0, 4096, s));
    const size_t lds = sizeof(float) * ((size_t)U * (NW * H + 4) +
                                        std::max(4 * (size_t)p.Npad * 16, (size_t)2 * N * U * NW));
    const dim3 grid(dirs * p.nwg);
    {
      ProfSpan ps(s, "rnn_bwd_rec");
      launch_rec(false, d.mode, p, grid, lds, s);
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
