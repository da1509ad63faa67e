// ctc.hip -- CTC loss and gradient for MI355X (gfx950), behind the warp-ctc C ABI
// (include/ctc.h).  Replaces warp-ctc's compute_ctc_loss as called from
// src/ctc/ctc-nnet-update.cc:211-243 of the reference.
//
// Three launches per call, all stream-ordered:
//   K1 ctc_logz        one wave per frame row: logZ[t,n] = logsumexp_a act[t,n,a]
//                      and lp[t,n,a] = act - logZ (fully parallel, HBM-bound:
//                      4*A B read + 4*A B written per row).
//   K2 ctc_alpha_beta  one workgroup per (utterance, direction): log-space
//                      alpha (forward) or beta (backward) recursion, serial
//                      over T with ONE workgroup barrier per group of 8 frames
//                      (ctc_alpha_beta_win: overlapping per-wave state windows,
//                      the default up to 600 extended labels; ab_body: 512
//                      threads with halo lanes, 1..3 states per thread).  The
//                      extended (blank-interleaved) label sequence lives in
//                      registers, the previous frame's column in double-buffered
//                      LDS, the emission log-probs (normalised by K1) are
//                      gathered into LDS a chunk of frames ahead by LDS-DMA.  Each frame is renormalised by the max of
//                      the previous column (wave max via DPP/shfl, then LDS) and
//                      the running offset is kept in fp64, so exp(alpha+beta-logp)
//                      keeps ~1e-7 relative accuracy at T=2000 (plain fp32 log
//                      space -- warp-ctc's own arithmetic -- loses ~1e-3).  The
//                      normalised columns are spilled to HBM (4*T*S B each).
//   K3 ctc_grad        (utterance, 8-frame chunk) per workgroup, fully parallel:
//                      gamma_t(k) = sum_{s: l'_s = k} exp(a~+b~+off), then
//                      grad = softmax - gamma; padding / infeasible rows get 0.
//                      Deterministic (fixed summation order, no atomics).
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <atomic>
#include <vector>

#include "common.h"
#include "ctc.h"
#include "prof.h"

namespace kctc {
namespace ctcimpl {

constexpr int kMaxLabel = 639;  // MAX_WARPCTC_LABEL_LENGTH, src/ctc/ctc-nnet-train.cc:25-26
constexpr int kThreads = 256;  // K3
constexpr int kABThreads = 512;  // K2: 8 waves, 2 per SIMD, <= 3 states per thread
constexpr int kABWaves = kABThreads / 64;
constexpr int kSPT = (2 * kMaxLabel + 1 + kABThreads - 1) / kABThreads;  // states per thread (3)
constexpr int kFR = 8;   // frames per K3 workgroup

struct UttDesc {
  int T, L, S, feasible, lab_off, pad;
  long long ab_off;   // float offset of this utterance's alpha spill; beta follows at +T*S
  long long off_off;  // double offset of offA[T]; offB follows at +T
};

struct Layout {
  size_t desc, labels, links, owner, costs, logz, lp, spill, offs, total;
  int T_max;
  long long spill_floats, off_doubles;
};

static bool make_layout(const int *label_lengths, const int *input_lengths, int A, int N,
                        Layout *lay, std::vector<UttDesc> *descs, bool *bad) {
  *bad = false;
  if (A <= 0 || N <= 0 || !label_lengths || !input_lengths) { *bad = true; return false; }
  int T_max = 0;
  long long nlab = 0, spill = 0, offs = 0;
  if (descs) descs->resize(N);
  for (int n = 0; n < N; n++) {
    int T = input_lengths[n], L = label_lengths[n];
    if (T < 0 || L < 0 || L > kMaxLabel) { *bad = true; return false; }
    T_max = T > T_max ? T : T_max;
    int S = 2 * L + 1;
    if (descs) {
      UttDesc &d = (*descs)[n];
      d.T = T; d.L = L; d.S = S; d.feasible = 0; d.lab_off = (int)nlab; d.pad = 0;
      d.ab_off = spill; d.off_off = offs;
    }
    nlab += L;
    spill += 2LL * T * S;
    offs += 2LL * T;
  }
  Layout &l = *lay;
  size_t p = 0;
  l.desc = p;   p = align_up(p + sizeof(UttDesc) * N, 256);
  l.labels = p; p = align_up(p + sizeof(int) * (nlab > 0 ? nlab : 1), 256);
  l.links = p;  p = align_up(p + sizeof(int) * (nlab > 0 ? nlab : 1), 256);  // next position of the same label
  l.owner = p;  p = align_up(p + sizeof(int) * (size_t)N * A, 256);          // first position of each label
  l.costs = p;  p = align_up(p + sizeof(double) * N, 256);
  l.logz = p;   p = align_up(p + sizeof(float) * (size_t)T_max * N + 4, 256);
  l.lp = p;     p = align_up(p + sizeof(float) * (size_t)T_max * N * A + 4, 256);
  l.spill = p;  p = align_up(p + sizeof(float) * (size_t)spill, 256);
  l.offs = p;   p = align_up(p + sizeof(double) * (size_t)offs, 256);
  l.total = p;
  l.T_max = T_max;
  l.spill_floats = spill;
  l.off_doubles = offs;
  return true;
}

// ---------------------------------------------------------------------------
// K1: per-frame log normaliser.  One wave per row, 4 rows per workgroup.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ctc_logz(const float *__restrict__ acts, int A, long rows,
                                                float *__restrict__ logz, float *__restrict__ lp) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float *r = acts + row * A;
  float m = -INFINITY;
  for (int a = lane; a < A; a += kWave) m = fmaxf(m, r[a]);
  m = wave_max(m);
  float s = 0.f;
  for (int a = lane; a < A; a += kWave) s += expf(r[a] - m);
  s = wave_sum(s);
  const float z = m + logf(s);
  if (lane == 0) logz[row] = z;
  for (int a = lane; a < A; a += kWave) lp[row * A + a] = r[a] - z;  // normalised log-probs (K2 input)
}

// log(e^a + e^b + e^c) as max + log1p(sum of the two smaller terms): the
// dominant term contributes exactly 1, so log1p keeps full relative precision
// of the small ones (logf(1 + x) would round x to the ulp of 1).  log1p(x) is
// evaluated as log(u) - ((u - 1) - x) with u = fl(1 + x): (u - 1) - x is
// u's rounding error, exact in fp32, and log(u) - c differs from log(u - c) by
// c (u - 1) / u, below 2^-24 of the result (u == 1 gives x exactly).  One
// hardware v_log_f32 (u in [1, 3]: no range reduction) and no reciprocal.
__device__ __forceinline__ float fast_log1p(float x) {
  const float u = 1.f + x;
  return __builtin_fmaf(__builtin_amdgcn_logf(u), 0.693147180559945309f, x - (u - 1.f));
}
// branch-free: -inf in, -inf out (all three -inf gives m = -inf, and
// -inf - -inf = NaN is selected away)
__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  const float lo = fminf(a, fminf(b, c));
  const float md = fmaxf(fminf(a, b), fminf(fmaxf(a, b), c));  // median, exact
  const float r = m + fast_log1p(__expf(md - m) + __expf(lo - m));
  return m == -INFINITY ? -INFINITY : r;
}

// ---------------------------------------------------------------------------
// K2: alpha (blockIdx.x < N) and beta (blockIdx.x >= N) recursions.
// ---------------------------------------------------------------------------
// The emission log-probs lp[t, n, l'_s] of the next chunk of F frames are
// gathered into LDS by LDS-DMA (global_load_lds, one 4-byte gather per lane
// and state block) while the current chunk is processed, so the serial frame
// loop itself issues no global load: per frame it reads LDS, computes, spills
// its column and meets ONE raw s_barrier (lgkmcnt only -- a __syncthreads()
// would drain the in-flight DMA).  The chunk's DMA is waited for once, at the
// chunk boundary.  All LDS is one dynamic array (a second __shared__ object
// makes hipcc wait vmcnt(0) before LDS reads while a DMA is in flight):
//   emit[2][F][SP] | col[2][CP] | wmax[2][8] | feasible flag
struct AbLds {
  int F, SP, CP;
  int pair;  // frames per barrier (SPT == 1, 1..8): mictc_set_frame_group
  __device__ __host__ size_t floats() const { return 2 * (size_t)F * SP + 2 * (size_t)CP + 2 * kABWaves + 4; }
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// the direction is a template parameter of the body: one code path per
// direction, so the scheduler is free to hoist each frame's LDS reads
template <bool SPILL, int SPT, bool is_beta>
__device__ __forceinline__ void ab_body(
    const float *__restrict__ lp, int N, int A, int blank, UttDesc *__restrict__ descs,
    const int *__restrict__ labels, float *__restrict__ spill, double *__restrict__ offs,
    double *__restrict__ costs, AbLds lay) {
  const int n = is_beta ? blockIdx.x - N : blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = lay.F, SP = lay.SP, CP = lay.CP;
  float *emit = lds;                       // [2][F][SP]
  float *colb = emit + 2 * (size_t)F * SP;  // [2][CP]
  float *wmax = colb + 2 * CP;             // [2][kABWaves]
  int *sh_feasible = reinterpret_cast<int *>(wmax + 2 * kABWaves);

  UttDesc d = descs[n];
  const int T = d.T, L = d.L, S = d.S;
  const int *lab = labels + d.lab_off;
  if (tid == 0) {
    int rep = 0;
    for (int i = 1; i < L; i++) rep += (lab[i] == lab[i - 1]);
    *sh_feasible = (T > 0 && L + rep <= T);
  }
  __syncthreads();
  const int feasible = *sh_feasible;
  if (!is_beta && tid == 0) {
    descs[n].feasible = feasible;
    if (!feasible) costs[n] = 0.0;
  }
  if (!feasible) return;

  // extended label of each owned state s = tid + 512 i, and its skip permission
  int ext[SPT];
  bool skip[SPT];
#pragma unroll
  for (int i = 0; i < SPT; i++) {
    int s = tid + i * kABThreads;
    ext[i] = (s < S) ? ((s & 1) ? lab[(s - 1) >> 1] : blank) : blank;
    skip[i] = false;
    if (s < S && (s & 1)) {
      if (!is_beta) skip[i] = (s >= 2) && (lab[(s - 1) >> 1] != lab[(s - 3) >> 1]);
      else skip[i] = (s + 2 < S) && (lab[(s + 1) >> 1] != lab[(s - 1) >> 1]);
    }
  }
  // beta: transition s -> s+2 allowed iff l'_{s+2} != blank and != l'_s; for
  // odd s that is lab[(s+1)/2] != lab[(s-1)/2]; for even s, l'_{s+2} is blank.

  // Groups of m frames per barrier (SPT == 1, m = lay.pair in 2..8): lanes
  // 0 .. 2(m-1)-1 of each wave also carry halo states of the neighbouring
  // wave -- alpha: 64 w - 2(m-1) .. 64 w - 1; beta: 64 w + 64 .. -- so frames
  // 2..m of a group need no exchange: their s - 1 / s - 2 (beta: s + 1 /
  // s + 2) come from the previous frame's values by wave shuffles, the halo
  // (shrinking by two states a frame) filling the wave edge.
  const int gm = SPT == 1 ? max(1, min(lay.pair, 8)) : 1;
  const int nh = 2 * (gm - 1);
  const int hs = is_beta ? 64 * wid + 64 + lane : 64 * wid - nh + lane;
  const bool hlive = lane < nh && hs >= 0 && hs < S;
  bool hskip = false;
  if (hlive && (hs & 1)) {
    if (!is_beta) hskip = (hs >= 2) && (lab[(hs - 1) >> 1] != lab[(hs - 3) >> 1]);
    else hskip = (hs + 2 < S) && (lab[(hs + 1) >> 1] != lab[(hs - 1) >> 1]);
  }
  const bool pair_ok = gm > 1;

  const long tstride = (long)N * A;
  const float *lrow = lp + (long)n * A;  // + t * N * A
  float *sp = spill + d.ab_off + (is_beta ? (long long)T * S : 0);
  double *op = offs + d.off_off + (is_beta ? T : 0);
  auto tframe = [&](int k) { return is_beta ? T - 1 - k : k; };  // k-th processed frame
  const int nblk = (S + 63) / 64;  // 64-state blocks; wave w gathers blocks w, w + 8, ...
  auto issue = [&](int c, int b) {
    float *dst = emit + (size_t)b * F * SP;
    for (int f = 0; f < F; f++) {
      const int k = c * F + f;
      if (k >= T) break;
      const float *src = lrow + (long)tframe(k) * tstride;
#pragma unroll
      for (int i = 0; i < SPT; i++) {
        const int sb = wid + kABWaves * i;
        if (sb < nblk) __builtin_amdgcn_global_load_lds(src + ext[i], dst + (size_t)f * SP + sb * 64, 4, 0, 0);
      }
    }
  };

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  double off = 0.0;
  int cur = 0;
  const int nchunk = (T + F - 1) / F;
  for (int c = 0; c < nchunk; c++) {
    if (c + 1 < nchunk) issue(c + 1, (c + 1) & 1);
    const float *em = emit + (size_t)(c & 1) * F * SP;
    const int fend = min(F, T - c * F);
    for (int f = 0; f < fend; f++) {
      const int k = c * F + f;
      const int t = tframe(k);
      if (pair_ok && k > 0 && f + 1 < fend) {
        // frames k .. k + g - 1 with one barrier; mu (the max of column k - 1)
        // renormalises frame k only
        const int g = min(gm, fend - f);
        const int sid = min(tid, SP - 1), hid = min(max(hs, 0), SP - 1);
        const float *wm = wmax + (cur ^ 1) * kABWaves;
        const float *pv = colb + (cur ^ 1) * CP;
        const int s0 = tid;
        float pa, pb, pc, ha, hb, hc;
        if (!is_beta) {
          pa = pv[min(s0, CP - 1)];
          pb = s0 >= 1 ? pv[max(s0 - 1, 0)] : -INFINITY;
          pc = skip[0] ? pv[max(s0 - 2, 0)] : -INFINITY;
          ha = pv[min(hid, CP - 1)];
          hb = hs >= 1 ? pv[min(max(hs - 1, 0), CP - 1)] : -INFINITY;
          hc = hskip ? pv[min(max(hs - 2, 0), CP - 1)] : -INFINITY;
        } else {
          pa = pv[min(s0, CP - 1)];
          pb = s0 + 1 < S ? pv[min(s0 + 1, CP - 1)] : -INFINITY;
          pc = skip[0] ? pv[min(s0 + 2, CP - 1)] : -INFINITY;
          ha = pv[min(hid, CP - 1)];
          hb = hs + 1 < S ? pv[min(hs + 1, CP - 1)] : -INFINITY;
          hc = hskip ? pv[min(hs + 2, CP - 1)] : -INFINITY;
        }
        float mu = wm[0];
#pragma unroll
        for (int w = 1; w < kABWaves; w++) mu = fmaxf(mu, wm[w]);
        off += (double)mu;
        float q = 0.f, hq = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          if (j >= g) break;
          const int tj = tframe(k + j);
          const float ly = em[(size_t)(f + j) * SP + sid];
          const float hly = em[(size_t)(f + j) * SP + hid];
          if (j > 0) {
            // the previous frame's values of s - 1, s - 2 (beta: s + 1, s + 2)
            // from the neighbouring lanes, the halo at the wave edge
            // whole-wave DPP shifts (wave_shr:1 / wave_shl:1); the edge lane
            // takes `old` -- the halo value broadcast by readlane
            constexpr int kShr1 = 0x138, kShl1 = 0x130;
            auto dpp = [](float old, float src, auto ctrl) {
              return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src),
                                                                decltype(ctrl)::value, 0xf, 0xf, false));
            };
            const int ninf = __float_as_int(-INFINITY);
            (void)ninf;
            if (!is_beta) {
              const float e1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hq), nh - 1));  // 64 w - 1
              const float e2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hq), nh - 2));  // 64 w - 2
              using R = std::integral_constant<int, kShr1>;
              const float b1 = dpp(e1, q, R{});   // lane l: q[l-1]; lane 0: 64 w - 1
              const float c1 = dpp(e2, b1, R{});  // lane l: q[l-2]; lane 1: 64 w - 1; lane 0: 64 w - 2
              const float g1 = dpp(-INFINITY, hq, R{}), g2 = dpp(-INFINITY, g1, R{});
              pa = q;
              pb = s0 >= 1 ? b1 : -INFINITY;
              pc = skip[0] ? c1 : -INFINITY;
              ha = hq;
              hb = hs >= 1 ? g1 : -INFINITY;
              hc = hskip ? g2 : -INFINITY;
            } else {
              const float e0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hq), 0));  // 64 w + 64
              const float e1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hq), 1));  // 64 w + 65
              using L = std::integral_constant<int, kShl1>;
              const float b1 = dpp(e0, q, L{});   // lane l: q[l+1]; lane 63: 64 w + 64
              const float c1 = dpp(e1, b1, L{});  // lane l: q[l+2]; lane 62: 64 w + 64; lane 63: 64 w + 65
              const float g1 = dpp(-INFINITY, hq, L{}), g2 = dpp(-INFINITY, g1, L{});
              pa = q;
              pb = s0 + 1 < S ? b1 : -INFINITY;
              pc = skip[0] ? c1 : -INFINITY;
              ha = hq;
              hb = lane + 1 < nh && hs + 1 < S ? g1 : -INFINITY;
              hc = lane + 2 < nh && hskip ? g2 : -INFINITY;
            }
          }
          const float m = j == 0 ? mu : 0.f;
          const float v = lse3(pa, pb, pc) - m;
          q = s0 < S ? v + ly : -INFINITY;
          hq = hlive ? (lse3(ha, hb, hc) - m) + hly : -INFINITY;
          if (SPILL && s0 < S) sp[(long)tj * S + s0] = is_beta ? v : q;
          if (tid == 0 && SPILL) op[tj] = off;
        }
        float *cc = colb + cur * CP;
        cc[s0] = q;
        float lm = wave_max_l63(q);
        if (lane == 63) wmax[cur * kABWaves + wid] = lm;
        lds_barrier();
        cur ^= 1;
        f += g - 1;
        continue;
      }
      float ly[SPT];
#pragma unroll
      for (int i = 0; i < SPT; i++) ly[i] = em[(size_t)f * SP + min(tid + i * kABThreads, SP - 1)];
      float *cc = colb + cur * CP;
      float lmax = -INFINITY;
      if (k == 0) {
        // init: alpha_0(0)=ly(blank), alpha_0(1)=ly(l1); beta_{T-1}(S-1)=beta(S-2)=0,
        // stored as q = beta + ly (the next step's input)
#pragma unroll
        for (int i = 0; i < SPT; i++) {
          int s = tid + i * kABThreads;
          if (s < S) {
            float v;
            if (!is_beta) v = (s <= 1) ? ly[i] : -INFINITY;
            else v = (s >= S - 2) ? 0.f : -INFINITY;
            if (SPILL) sp[(long)t * S + s] = v;
            float q = is_beta ? v + ly[i] : v;
            cc[s] = q;
            lmax = fmaxf(lmax, q);
          }
        }
      } else {
        // all LDS reads of the frame up front, branch-free (clamped indices,
        // -inf selected in); the previous column's max mu is only subtracted
        // at the end: lse3(a, b, c) - mu == lse3(a - mu, b - mu, c - mu)
        const float *wm = wmax + (cur ^ 1) * kABWaves;
        const float *pv = colb + (cur ^ 1) * CP;
        float pa[SPT], pb[SPT], pc[SPT];
#pragma unroll
        for (int i = 0; i < SPT; i++) {
          const int s = tid + i * kABThreads;
          if (!is_beta) {
            pa[i] = pv[min(s, CP - 1)];
            pb[i] = pv[max(s - 1, 0)];
            pc[i] = pv[max(s - 2, 0)];
            pb[i] = s >= 1 ? pb[i] : -INFINITY;
            pc[i] = skip[i] ? pc[i] : -INFINITY;
          } else {
            pa[i] = pv[min(s, CP - 1)];
            pb[i] = pv[min(s + 1, CP - 1)];
            pc[i] = pv[min(s + 2, CP - 1)];
            pb[i] = s + 1 < S ? pb[i] : -INFINITY;
            pc[i] = skip[i] ? pc[i] : -INFINITY;
          }
        }
        float mu = wm[0];
#pragma unroll
        for (int w = 1; w < kABWaves; w++) mu = fmaxf(mu, wm[w]);
        // every lane computes and writes (cc is padded to SPT * 512 entries;
        // states >= S only ever feed selects): no load is sunk into a branch,
        // so the frame's LDS reads share one wait
#pragma unroll
        for (int i = 0; i < SPT; i++) {
          const int s = tid + i * kABThreads;
          const float v = lse3(pa[i], pb[i], pc[i]) - mu;
          const float q = v + ly[i];         // alpha: the new alpha~; beta: the next step's input
          const float spv = is_beta ? v : q;  // spilled: alpha~ / beta~
          cc[s] = q;
          lmax = fmaxf(lmax, s < S ? q : -INFINITY);
          if (SPILL && s < S) sp[(long)t * S + s] = spv;
        }
        off += (double)mu;
      }
      lmax = wave_max_l63(lmax);
      if (lane == 63) wmax[cur * kABWaves + wid] = lmax;
      if (tid == 0 && SPILL) op[t] = off;
      lds_barrier();
      cur ^= 1;
    }
    // the next chunk's gathers have landed; every wave is done with this chunk's buffer
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  }
  if (!is_beta && tid == 0) {
    // log p = O_{T-1} + lse(alpha~_{T-1}(S-1), alpha~_{T-1}(S-2))
    const float *pv = colb + (cur ^ 1) * CP;
    float a = pv[S - 1], b = S > 1 ? pv[S - 2] : -INFINITY;
    float m = fmaxf(a, b);
    double lpv = off + (double)m + log((double)expf(a - m) + (double)expf(b - m));
    costs[n] = -lpv;
  }
}

// ---------------------------------------------------------------------------
// K2, overlapping windows (S <= kWinWaves x own states; the default path).
// Frames go in groups of m per barrier as in ab_body, but instead of a second
// log-sum-exp per lane for the halo, each wave's 64 lanes hold a WINDOW of 64
// consecutive states: `own` = 64 - 2 (m - 1) of them its own, the other
// 2 (m - 1) the neighbour's edge (alpha: the states below, beta: above).
// Within a group the previous frame's s - 1 / s - 2 (beta: s + 1 / s + 2) come
// from the neighbouring lanes by whole-wave DPP shifts; the lanes a shift
// cannot feed (the window's far edge) go stale by two per frame, which after
// m - 1 frames reaches exactly the halo, so every own state stays exact and
// every lane computes ONE log-sum-exp per frame.  The group's first frame
// reads the whole previous column from LDS (own states written by their
// waves at the group's end) and carries the renormalisation.  Same spill,
// offsets and costs as ab_body; more waves (ceil(S / own), up to 12 at m = 8).
constexpr int kWinWaves = 12;
template <bool SPILL, bool is_beta>
__device__ __forceinline__ void win_body(const float *__restrict__ lp, int N, int A, int blank,
                                         UttDesc *__restrict__ descs, const int *__restrict__ labels,
                                         float *__restrict__ spill, double *__restrict__ offs,
                                         double *__restrict__ costs, AbLds lay) {
  const int n = is_beta ? blockIdx.x - N : blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nwv = blockDim.x >> 6;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = lay.F, SP = lay.SP, CP = lay.CP;
  float *emit = lds;                        // [2][F][SP]
  float *colb = emit + 2 * (size_t)F * SP;  // [2][CP]
  float *wmax = colb + 2 * CP;              // [2][kWinWaves]
  int *sh_feasible = reinterpret_cast<int *>(wmax + 2 * kWinWaves);

  UttDesc d = descs[n];
  const int T = d.T, L = d.L, S = d.S;
  const int *lab = labels + d.lab_off;
  if (tid == 0) {
    int rep = 0;
    for (int i = 1; i < L; i++) rep += (lab[i] == lab[i - 1]);
    *sh_feasible = (T > 0 && L + rep <= T);
  }
  __syncthreads();
  const int feasible = *sh_feasible;
  if (!is_beta && tid == 0) {
    descs[n].feasible = feasible;
    if (!feasible) costs[n] = 0.0;
  }
  if (!feasible) return;

  const int gm = max(1, min(lay.pair, 8)), nh = 2 * (gm - 1), own = 64 - nh;
  const int s = is_beta ? own * wid + lane : own * wid - nh + lane;  // this lane's state
  const bool mine = is_beta ? lane < own : lane >= nh;
  const bool live = s >= 0 && s < S;
  bool skip = false;  // alpha: s - 2 -> s allowed; beta: s + 2 -> s (see ab_body)
  if (live && (s & 1)) {
    if (!is_beta) skip = (s >= 2) && (lab[(s - 1) >> 1] != lab[(s - 3) >> 1]);
    else skip = (s + 2 < S) && (lab[(s + 1) >> 1] != lab[(s - 1) >> 1]);
  }
  const int sc = min(max(s, 0), CP - 1);  // clamped LDS index
  auto at = [&](int x) { return min(max(x, 0), CP - 1); };
  // emission gather: wave w fills state block w (nwv >= ceil(S / 64) blocks)
  const int nblk = (S + 63) / 64, gs = wid * 64 + lane;
  const int gext = gs < S ? ((gs & 1) ? lab[(gs - 1) >> 1] : blank) : blank;
  const long tstride = (long)N * A;
  const float *lrow = lp + (long)n * A;
  float *sp = spill + d.ab_off + (is_beta ? (long long)T * S : 0);
  double *op = offs + d.off_off + (is_beta ? T : 0);
  auto tframe = [&](int k) { return is_beta ? T - 1 - k : k; };
  auto issue = [&](int c, int b) {
    if (wid >= nblk) return;
    float *dst = emit + (size_t)b * F * SP + wid * 64;
    for (int f = 0; f < F; f++) {
      const int k = c * F + f;
      if (k >= T) break;
      __builtin_amdgcn_global_load_lds(lrow + (long)tframe(k) * tstride + gext, dst + (size_t)f * SP, 4, 0, 0);
    }
  };
  const int ems = min(max(s, 0), SP - 1);
  auto publish = [&](int cur, float q) {  // own states of the column, the wave's max, barrier
    if (mine && s < CP) colb[cur * CP + s] = q;
    const float lm = wave_max_l63(mine && live ? q : -INFINITY);
    if (lane == 63) wmax[cur * kWinWaves + wid] = lm;
    lds_barrier();
  };

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  double off = 0.0;
  int cur = 0;
  float q = -INFINITY;
  const int nchunk = (T + F - 1) / F;
  for (int c = 0; c < nchunk; c++) {
    if (c + 1 < nchunk) issue(c + 1, (c + 1) & 1);
    const float *em = emit + (size_t)(c & 1) * F * SP;
    const int fend = min(F, T - c * F);
    int f = 0;
    if (c == 0) {
      // init: alpha_0(0) = ly(blank), alpha_0(1) = ly(l1); beta_{T-1}(S-1) =
      // beta(S-2) = 0, kept as q = beta + ly (the next step's input)
      const int t = tframe(0);
      const float ly = em[ems];
      const float v = !live ? -INFINITY : !is_beta ? (s <= 1 ? ly : -INFINITY) : (s >= S - 2 ? 0.f : -INFINITY);
      q = live ? (is_beta ? v + ly : v) : -INFINITY;
      if (SPILL && mine && live) sp[(long)t * S + s] = v;
      if (SPILL && tid == 0) op[t] = off;
      publish(cur, q);
      cur ^= 1;
      f = 1;
    }
    while (f < fend) {
      const int g = min(gm, fend - f), k = c * F + f;
      const float *pv = colb + (cur ^ 1) * CP;
      const float *wm = wmax + (cur ^ 1) * kWinWaves;
      float pa = pv[sc], pb, pc;
      if (!is_beta) {
        pb = s >= 1 ? pv[at(s - 1)] : -INFINITY;
        pc = skip ? pv[at(s - 2)] : -INFINITY;
      } else {
        pb = s + 1 < S ? pv[at(s + 1)] : -INFINITY;
        pc = skip ? pv[at(s + 2)] : -INFINITY;
      }
      float mu = wm[0];
      for (int w = 1; w < nwv; w++) mu = fmaxf(mu, wm[w]);
      off += (double)mu;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (j >= g) break;
        const int t = tframe(k + j);
        const float ly = em[(size_t)(f + j) * SP + ems];
        if (j > 0) {
          // whole-wave DPP shifts: alpha wave_shr:1 (lane l <- q[l - 1]),
          // beta wave_shl:1 (lane l <- q[l + 1]); the edge lane gets -inf
          constexpr int ctrl = is_beta ? 0x130 : 0x138;
          const int ninf = __float_as_int(-INFINITY);
          const float b1 = __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(q), ctrl, 0xf, 0xf, false));
          const float c1 = __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(b1), ctrl, 0xf, 0xf, false));
          pa = q;
          pb = (is_beta ? s + 1 < S : s >= 1) ? b1 : -INFINITY;
          pc = skip ? c1 : -INFINITY;
        }
        const float v = lse3(pa, pb, pc) - (j == 0 ? mu : 0.f);
        q = live ? v + ly : -INFINITY;
        if (SPILL && mine && live) sp[(long)t * S + s] = is_beta ? v : q;
        if (SPILL && tid == 0) op[t] = off;
      }
      publish(cur, q);
      cur ^= 1;
      f += g;
    }
    // the next chunk's gathers have landed; every wave is done with this chunk's buffer
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  }
  if (!is_beta && tid == 0) {
    // log p = O_{T-1} + lse(alpha~_{T-1}(S-1), alpha~_{T-1}(S-2))
    const float *pv = colb + (cur ^ 1) * CP;
    float a = pv[S - 1], b = S > 1 ? pv[S - 2] : -INFINITY;
    float m = fmaxf(a, b);
    double lpv = off + (double)m + log((double)expf(a - m) + (double)expf(b - m));
    costs[n] = -lpv;
  }
}

template <bool SPILL>
__global__ __launch_bounds__(64 * kWinWaves) void ctc_alpha_beta_win(
    const float *__restrict__ lp, int N, int A, int blank, UttDesc *__restrict__ descs,
    const int *__restrict__ labels, float *__restrict__ spill, double *__restrict__ offs,
    double *__restrict__ costs, AbLds lay) {
  if (blockIdx.x >= (unsigned)N) win_body<SPILL, true>(lp, N, A, blank, descs, labels, spill, offs, costs, lay);
  else win_body<SPILL, false>(lp, N, A, blank, descs, labels, spill, offs, costs, lay);
}

template <bool SPILL, int SPT>
__global__ __launch_bounds__(kABThreads) void ctc_alpha_beta(
    const float *__restrict__ lp, int N, int A, int blank, UttDesc *__restrict__ descs,
    const int *__restrict__ labels, float *__restrict__ spill, double *__restrict__ offs,
    double *__restrict__ costs, AbLds lay) {
  if (blockIdx.x >= (unsigned)N) ab_body<SPILL, SPT, true>(lp, N, A, blank, descs, labels, spill, offs, costs, lay);
  else ab_body<SPILL, SPT, false>(lp, N, A, blank, descs, labels, spill, offs, costs, lay);
}

// ---------------------------------------------------------------------------
// K3: gradient.  grid (ceil(T_max/FR), N), 256 threads.
// dynamic LDS: occ[FR][S] | next[L] | owner[A] | gblank[FR] | gtot[FR]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void ctc_grad(
    const float *__restrict__ acts, const float *__restrict__ logz, float *__restrict__ grads,
    int N, int A, int T_max, int blank, const UttDesc *__restrict__ descs,
    const int *__restrict__ links, const int *__restrict__ owners, const float *__restrict__ spill,
    const double *__restrict__ offs, const double *__restrict__ costs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.y, t0 = blockIdx.x * kFR, tid = threadIdx.x;
  const UttDesc d = descs[n];
  const int T = d.feasible ? d.T : 0, L = d.L, S = d.S;
  const int nf = min(kFR, T_max - t0);
  if (t0 >= T) {  // padding or infeasible: zero rows
    for (int it = tid; it < nf * A; it += kThreads) {
      int f = it / A, a = it - f * A;
      grads[((long)(t0 + f) * N + n) * A + a] = 0.f;
    }
    return;
  }
  float *occ = reinterpret_cast<float *>(smem);
  int *nxt = reinterpret_cast<int *>(occ + kFR * S);
  int *owner = nxt + (L > 0 ? L : 1);
  float *gblank = reinterpret_cast<float *>(owner + A);
  float *gtot = gblank + kFR;
  // label chains (first position of each label, next position of the same
  // label), computed once per call on the host and staged with the labels
  for (int a = tid; a < A; a += kThreads) owner[a] = owners[(long)n * A + a];
  for (int j = tid; j < L; j += kThreads) nxt[j] = links[d.lab_off + j];
  const double logp = -costs[n];
  const float *al = spill + d.ab_off;
  const float *be = al + (long long)T * S;
  const double *oa = offs + d.off_off, *ob = oa + T;
  const int nreal = min(nf, T - t0);
  for (int f = 0; f < nreal; f++) {
    const int t = t0 + f;
    const float Kt = (float)(oa[t] + ob[t] - logp);
    for (int s = tid; s < S; s += kThreads) {
      float v = al[(long)t * S + s] + be[(long)t * S + s];
      occ[f * S + s] = (v == -INFINITY) ? 0.f : expf(v + Kt);
    }
  }
  __syncthreads();
  // blank occupancy and total occupancy: wave w sums frames w, w+4.  gamma is
  // normalised by the frame's own total sum_s alpha_t(s) beta_t(s) (= p for
  // every t): the alpha and beta rounding accumulated over T steps is common
  // to every state of a frame and cancels, instead of surviving against logp.
  {
    const int lane = tid & 63, wid = tid >> 6;
    for (int f = wid; f < nreal; f += kThreads / kWave) {
      float acc = 0.f, tot = 0.f;
      for (int s = 2 * lane; s < S; s += 2 * kWave) {
        acc += occ[f * S + s];
        tot += occ[f * S + s] + (s + 1 < S ? occ[f * S + s + 1] : 0.f);
      }
      acc = wave_sum(acc);
      tot = wave_sum(tot);
      if (lane == 0) { gblank[f] = acc / tot; gtot[f] = 1.f / tot; }
    }
  }
  __syncthreads();
  for (int it = tid; it < nf * A; it += kThreads) {
    const int f = it / A, a = it - f * A, t = t0 + f;
    const long idx = ((long)t * N + n) * A + a;
    float g = 0.f;
    if (t < T) {
      float gam = 0.f;
      if (a == blank) {
        gam = gblank[f];
      } else {
        for (int j = owner[a]; j >= 0; j = nxt[j]) gam += occ[f * S + 2 * j + 1];
        gam *= gtot[f];
      }
      g = expf(acts[idx] - logz[(long)t * N + n]) - gam;
    }
    grads[idx] = g;
  }
}

struct Staging {
  char *buf = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};
static thread_local Staging g_stage;

static char *staging_acquire(size_t bytes) {
  Staging &s = g_stage;
  if (s.pending) {
    if (hipEventSynchronize(s.ev) != hipSuccess) return nullptr;
    s.pending = false;
  }
  if (!s.ev && hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) return nullptr;
  if (bytes > s.cap) {
    if (s.buf) (void)hipHostFree(s.buf);
    size_t cap = align_up(bytes * 2, 4096);
    if (hipHostMalloc((void **)&s.buf, cap, hipHostMallocDefault) != hipSuccess) {
      s.buf = nullptr; s.cap = 0;
      return nullptr;
    }
    s.cap = cap;
  }
  return s.buf;
}
static void staging_release(hipStream_t stream) {
  if (hipEventRecord(g_stage.ev, stream) == hipSuccess) g_stage.pending = true;
}

// frames per barrier of ctc_alpha_beta (mictc_set_frame_group)
static std::atomic<int> g_frame_group{0};
static int frame_group() {
  int m = g_frame_group.load(std::memory_order_relaxed);
  if (m <= 0) {
    m = 8;
    int expect = 0;
    g_frame_group.compare_exchange_strong(expect, m);
    m = g_frame_group.load(std::memory_order_relaxed);
  }
  return m;
}

// the overlapping-window alpha / beta kernel (default; mictc_set_win(0): the
// 512-thread ab_body kernel with halo log-sum-exps, as before round 6)
static std::atomic<int> g_win{1};
static bool win_enabled() { return g_win.load(std::memory_order_relaxed) != 0; }

static ctcStatus_t launch(const float *acts, float *grads, const int *flat_labels,
                          const int *label_lengths, const int *input_lengths, int A, int N,
                          double *costs_dev, void *workspace, hipStream_t stream, int blank) {
  Layout lay;
  std::vector<UttDesc> descs;
  bool bad = false;
  if (!make_layout(label_lengths, input_lengths, A, N, &lay, &descs, &bad) || bad)
    return CTC_STATUS_INVALID_VALUE;
  if (blank < 0 || blank >= A || !acts || !workspace) return CTC_STATUS_INVALID_VALUE;
  long long nlab = 0;
  for (int n = 0; n < N; n++) nlab += label_lengths[n];
  for (long long i = 0; i < nlab; i++)
    if (flat_labels[i] < 0 || flat_labels[i] >= A || flat_labels[i] == blank)
      return CTC_STATUS_INVALID_VALUE;
  char *ws = static_cast<char *>(workspace);
  // host staging (pinned, reused once the previous call's copy has landed):
  // descriptors then labels, one H2D copy
  char *stage = staging_acquire(lay.costs);
  if (!stage) return CTC_STATUS_MEMOPS_FAILED;
  memcpy(stage + lay.desc, descs.data(), sizeof(UttDesc) * N);
  if (nlab) memcpy(stage + lay.labels, flat_labels, sizeof(int) * nlab);
  {
    // per utterance: owner[a] = first position of label a (-1: absent),
    // links[j] = next position holding the same label as j (-1: last)
    int *links = reinterpret_cast<int *>(stage + lay.links), *owner = reinterpret_cast<int *>(stage + lay.owner);
    std::fill(owner, owner + (size_t)N * A, -1);
    long long off = 0;
    for (int n = 0; n < N; n++) {
      const int L = label_lengths[n];
      int *own = owner + (size_t)n * A;
      for (int j = L - 1; j >= 0; j--) {
        const int k = flat_labels[off + j];
        links[off + j] = own[k];
        own[k] = j;
      }
      off += L;
    }
  }
  if (hipMemcpyAsync(ws, stage, lay.costs, hipMemcpyHostToDevice, stream) != hipSuccess)
    return CTC_STATUS_MEMOPS_FAILED;
  staging_release(stream);
  UttDesc *d_desc = reinterpret_cast<UttDesc *>(ws + lay.desc);
  const int *d_lab = reinterpret_cast<const int *>(ws + lay.labels);
  float *d_logz = reinterpret_cast<float *>(ws + lay.logz);
  float *d_spill = reinterpret_cast<float *>(ws + lay.spill);
  double *d_offs = reinterpret_cast<double *>(ws + lay.offs);
  const long rows = (long)lay.T_max * N;
  float *d_lp = reinterpret_cast<float *>(ws + lay.lp);
  if (rows > 0) {
    ProfSpan ps(stream, "ctc_logz");
    hipLaunchKernelGGL(ctc_logz, dim3(ceil_div(rows, 4)), dim3(256), 0, stream, acts, A, rows,
                       d_logz, d_lp);
  }
  const int want = grads != nullptr;
  {
    int Smax = 1;
    for (int n = 0; n < N; n++) Smax = 2 * label_lengths[n] + 1 > Smax ? 2 * label_lengths[n] + 1 : Smax;
    AbLds al;
    al.pair = frame_group();  // measured: 8 < 6 < 4 < 3 < 1 < 2 (ms)
    al.SP = (Smax + 63) / 64 * 64;
    // overlapping windows (ctc_alpha_beta_win) up to kWinWaves waves
    const int own = 64 - 2 * (std::max(1, std::min(al.pair, 8)) - 1);
    const int nwv = std::max(1, (Smax + own - 1) / own);
    if (nwv <= kWinWaves && win_enabled()) {
      al.CP = std::max((Smax + 4 + 3) / 4 * 4, own * nwv);
      al.F = (int)std::min<size_t>(32, std::max<size_t>(4, (size_t)96 * 1024 / (2 * sizeof(float) * al.SP)));
      const size_t shm = sizeof(float) * (2 * (size_t)al.F * al.SP + 2 * (size_t)al.CP + 2 * kWinWaves + 4);
      if (shm > 160 * 1024) return CTC_STATUS_INVALID_VALUE;
      ProfSpan ps(stream, "ctc_alpha_beta");
      auto kern = want ? ctc_alpha_beta_win<true> : ctc_alpha_beta_win<false>;
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm);
      hipLaunchKernelGGL(kern, dim3(want ? 2 * N : N), dim3(64 * nwv), shm, stream, d_lp, N, A, blank, d_desc, d_lab,
                         d_spill, d_offs, costs_dev, al);
    } else {
      al.CP = std::max((Smax + 4 + 3) / 4 * 4, (Smax <= kABThreads ? 1 : kSPT) * kABThreads);
      // chunk depth: as many frames as fit 96 KB of double-buffered emissions (4..32)
      al.F = (int)std::min<size_t>(32, std::max<size_t>(4, (size_t)96 * 1024 / (2 * sizeof(float) * al.SP)));
      const size_t shm = sizeof(float) * al.floats();
      if (shm > 160 * 1024) return CTC_STATUS_INVALID_VALUE;
      ProfSpan ps(stream, "ctc_alpha_beta");
      auto go = [&](auto kern, int grid) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)shm);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kABThreads), shm, stream, d_lp, N, A, blank, d_desc, d_lab,
                           d_spill, d_offs, costs_dev, al);
      };
      // one state per thread up to 512 extended labels (L <= 255), else three
      if (Smax <= kABThreads) {
        if (want) go(ctc_alpha_beta<true, 1>, 2 * N);
        else go(ctc_alpha_beta<false, 1>, N);
      } else {
        if (want) go(ctc_alpha_beta<true, kSPT>, 2 * N);
        else go(ctc_alpha_beta<false, kSPT>, N);
      }
    }
  }
  if (want && lay.T_max > 0) {
    int Lmax = 0;
    for (int n = 0; n < N; n++) Lmax = label_lengths[n] > Lmax ? label_lengths[n] : Lmax;
    const int Smax = 2 * Lmax + 1;
    size_t shm = sizeof(float) * kFR * Smax + sizeof(int) * (Lmax > 0 ? Lmax : 1) +
                 sizeof(int) * A + 2 * sizeof(float) * kFR;
    if (shm > 160 * 1024) return CTC_STATUS_INVALID_VALUE;
    ProfSpan ps(stream, "ctc_grad");
    hipLaunchKernelGGL(ctc_grad, dim3(ceil_div(lay.T_max, kFR), N), dim3(kThreads), shm, stream,
                       acts, d_logz, grads, N, A, lay.T_max, blank, d_desc,
                       reinterpret_cast<const int *>(ws + lay.links), reinterpret_cast<const int *>(ws + lay.owner),
                       d_spill, d_offs, costs_dev);
  }
  if (hipGetLastError() != hipSuccess) return CTC_STATUS_EXECUTION_FAILED;
  return CTC_STATUS_SUCCESS;
}

}  // namespace ctcimpl
}  // namespace kctc

using namespace kctc::ctcimpl;

extern "C" {

int get_warpctc_version(void) { return 2; }

int mictc_set_frame_group(int m) {
  const int prev = frame_group();
  if (m > 0) g_frame_group.store(std::max(1, std::min(m, 8)));
  return prev;
}

int mictc_set_win(int on) {
  const int prev = g_win.load();
  if (on >= 0) g_win.store(on ? 1 : 0);
  return prev;
}

const char *ctcGetStatusString(ctcStatus_t status) {
  switch (status) {
    case CTC_STATUS_SUCCESS: return "no error";
    case CTC_STATUS_MEMOPS_FAILED: return "cuda memcpy or memset failed";
    case CTC_STATUS_INVALID_VALUE: return "invalid value";
    case CTC_STATUS_EXECUTION_FAILED: return "execution failed";
    case CTC_STATUS_UNKNOWN_ERROR:
    default: return "unknown error";
  }
}

ctcStatus_t get_workspace_size(const int *const label_lengths, const int *const input_lengths,
                               int alphabet_size, int minibatch, struct ctcOptions info,
                               size_t *size_bytes) {
  if (!size_bytes || info.loc != CTC_GPU) return CTC_STATUS_INVALID_VALUE;
  Layout lay;
  bool bad = false;
  if (!make_layout(label_lengths, input_lengths, alphabet_size, minibatch, &lay, nullptr, &bad) ||
      bad)
    return CTC_STATUS_INVALID_VALUE;
  *size_bytes = lay.total;
  return CTC_STATUS_SUCCESS;
}

ctcStatus_t mictc_compute_ctc_loss_async(const float *activations, float *gradients,
                                         const int *flat_labels, const int *label_lengths,
                                         const int *input_lengths, int alphabet_size,
                                         int minibatch, double *costs_dev, void *workspace,
                                         ctcStream_t stream, int blank_label) {
  if (!costs_dev) return CTC_STATUS_INVALID_VALUE;
  try {
    return launch(activations, gradients, flat_labels, label_lengths, input_lengths,
                  alphabet_size, minibatch, costs_dev, workspace,
                  reinterpret_cast<hipStream_t>(stream), blank_label);
  } catch (...) {
    return CTC_STATUS_UNKNOWN_ERROR;
  }
}

ctcStatus_t compute_ctc_loss(const float *const activations, float *gradients,
                             const int *const flat_labels, const int *const label_lengths,
                             const int *const input_lengths, int alphabet_size, int minibatch,
                             float *costs, void *workspace, struct ctcOptions options) {
  if (options.loc != CTC_GPU || !costs) return CTC_STATUS_INVALID_VALUE;
  Layout lay;
  bool bad = false;
  if (!make_layout(label_lengths, input_lengths, alphabet_size, minibatch, &lay, nullptr, &bad) ||
      bad)
    return CTC_STATUS_INVALID_VALUE;
  hipStream_t stream = reinterpret_cast<hipStream_t>(options.stream);
  double *d_costs = reinterpret_cast<double *>(static_cast<char *>(workspace) + lay.costs);
  ctcStatus_t st = mictc_compute_ctc_loss_async(activations, gradients, flat_labels,
                                                label_lengths, input_lengths, alphabet_size,
                                                minibatch, d_costs, workspace, options.stream,
                                                options.blank_label);
  if (st != CTC_STATUS_SUCCESS) return st;
  std::vector<double> hc(minibatch);
  if (hipMemcpyAsync(hc.data(), d_costs, sizeof(double) * minibatch, hipMemcpyDeviceToHost,
                     stream) != hipSuccess)
    return CTC_STATUS_MEMOPS_FAILED;
  if (hipStreamSynchronize(stream) != hipSuccess) return CTC_STATUS_EXECUTION_FAILED;
  for (int n = 0; n < minibatch; n++) costs[n] = (float)hc[n];
  return CTC_STATUS_SUCCESS;
}

}  // extern "C"
