// gemm_x3p.hip -- split-fp16 GEMM on pre-packed operands (gfx950).
//
// The fp32-class product of gemm.hip's x3 kernel, with the fp32 -> (hi, lo)
// conversion moved out of the GEMM's staging path into pack passes that run
// once per operand:
//
//   packed operand P[r][kb][64] (fp16): the 32 values k = 32 kb .. 32 kb + 31
//   of row r, scaled by 2^e[r], as 32 hi halves then 32 lo halves (128 B);
//   e[r] puts the row's max |x| in [2^13, 2^14) (or comes from a bound on |x|).
//
// C[m][n] = alpha * 2^-(eA[m] + eB[n]) * sum_k (Ahi Bhi + Ahi Blo + Alo Bhi)
//           (+ beta C + bias), both operands packed along K.
//
// The GEMM is a plain fp16 matrix-core kernel: 128 x 128 tile, 4 waves (2 x 2,
// 64 x 64 each, 16 v_mfma_f32_16x16x32_f16 accumulators), one 32-k block per
// stage.  Stages are filled by LDS-DMA (global_load_lds_dwordx4, 16 B per
// lane): the LDS image of a tile is 128 rows x 128 B with the eight 16-B
// chunks of row r stored at chunk (c ^ (r & 7)) -- the swizzle is applied to
// the per-lane SOURCE address, so the DMA destination stays lane-linear -- and
// the fragment reads (ds_read_b128, rows fr = lane & 15, chunk fq or 4 + fq)
// are conflict-free.  Two stages in flight, one barrier per stage.
#include <algorithm>
#include <vector>

#include "common.h"
#include "gemm.h"

namespace kctc {
namespace {

constexpr int TB = 128;          // tile rows (M) = tile cols (N)
constexpr int NTH = 256;
constexpr int ROWB = 128;        // bytes per packed row block (64 halves)
constexpr int TILEB = TB * ROWB; // 16 KB per operand tile per stage
constexpr unsigned long long kWaitTicks = 300000000ull;  // streaming waits: 3 s of the 100 MHz clock
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

struct PParams {
  const _Float16 *A, *B;
  const int *eA, *eB;
  float *C;
  const float *bias, *bias2;
  long ldc;
  long sA, sB, sC, sBias, seA, seB;  // batch strides (A, B in halves; eA, eB in ints)
  int M, N, KB;
  int gx, tiles, batch, split, kbchunk;
  float alpha, beta;
  float *ws;
  int *counter;
  int eA0, eB0;
  const unsigned *sflags;  // streaming mode: producer flag lines
  int snwg, sT, sN;
  int srg;                 // producer row groups (flag lines and images per group)
  int sgsh;                // log2 of the sequences per row group (4: 16, 3: 8)
  int nrt;                 // row tiles
  long sxs;                // halves per producer step image
  long sxg;                // halves per row group's part of a step image
  int backoff;             // streaming waits sleep in proportion to the producer's distance
  int sdir;                // streaming: K split by producer direction (two half-K jobs per C tile, see fwd_combine)
  int dbg;                 // diagnostics (0 in the product): 1 no combine wait, 2 wait for both directions, 4 no combine,
                           // 32 register-A k loop without the two-deep prefetch
  unsigned *serr;          // producer's error word (wait timeout)
  int p256v;               // 256-tile k loop: 2 DMA spread over the MFMAs, 1 DMA block per stage, 0 auto
  const unsigned *xcd_word;  // XCDs of a pinned producer (X3PBwdStream::xcd_word), xcd_count of them
  int xcd_count;
  // backward stream (x3p_bwd_stream_kernel)
  const float *E;          // source rows of direction d: E + row * lde + d * edoff (KB * 32 floats)
  long lde, edoff;
  int P;                   // pack jobs per row tile
  int *done;               // [2][nrt] pack jobs finished
  int *arrive;             // [nrt][gx] direction partials arrived (+1) / partial published (+2)
  float *part;             // [M][N] the first direction's partial
  int mt;                  // row tiles
  const unsigned *avoid;   // X3PArgs::avoid_word, avoid_xcds
  int nxcd;
  // row stream (x3p_bwd_stream256_kernel) off a FORWARD producer: direction 0
  // frames ascending, direction 1 descending; bias + bias2 of column c at
  // (c / bcols) * sBias + c % bcols, added by the second partial
  int fwdp, bcols;
  // split-K tail: the last tailr row-tile slots of each direction (ready only
  // at the producer's last steps) run as tails K-splits each; their tiles'
  // partials meet in part2 ([tail tile][tails + 1][256 x 256])
  int tailr, tails;
  float *part2;
};


template <int AUX = 0>
__device__ __forceinline__ void issue_tile(const _Float16 *__restrict__ P, int rows, int r0, int KB, int kb,
                                           unsigned char *dst) {
  // wave w fills rows [32 w, 32 w + 32) of the tile: 4 instructions of 8 rows x 128 B
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int q = w * 4 + i;
    const int r = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int gr = r0 + r;
    gr = gr < rows ? gr : rows - 1;  // rows past the edge: any valid row (results discarded)
    const _Float16 *src = P + ((long)gr * KB + kb) * 64 + c * 8;
    __builtin_amdgcn_global_load_lds(src, dst + q * 1024, 16, 0, AUX);
  }
}

// streaming A operand: the producer's exchange images, read in place.  Step t
// of a bidirectional v6 forward recurrence holds h_t * 2^14 as fp16 hi/lo
// A fragments, [kb = k / 32][hi | lo][16 rows n][32 k] halves (kb over both
// directions), sxs halves per step; packed row r = t * sN + n.  The tile image
// is the same swizzled one as issue_tile's, filled by sc1 register loads (the
// rows were just published by other CUs) + ds_write_b128.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load_tile_xch(const PParams &p, const _Float16 *__restrict__ X, int r0, int kb,
                                              u32x4 (&reg)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(X), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int r = (w * 4 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = min(r0 + r, p.M - 1);
    const int t = gr / p.sN, n = gr - t * p.sN;
    const long off = (long)t * p.sxs + (long)(n >> p.sgsh) * p.sxg +
                     (((long)kb * 2 + (c >> 2)) * 16 + (n & ((1 << p.sgsh) - 1))) * 32 +
                     (c & 3) * 8;
    reg[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off * 2), 0, 16 /* sc1 */);
  }
}
// the packed layout [row][KB][64], rows written by other workgroups (sc1 stores):
// sc1 loads to registers, the tile image as issue_tile's
__device__ __forceinline__ void load_tile_sc1(const _Float16 *__restrict__ P, int rows, int r0, int KB, int kb,
                                              u32x4 (&reg)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int r = (w * 4 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = min(r0 + r, rows - 1);
    // one (uniform) descriptor: the host keeps rows * KB * 128 B below 2^31
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(P), 0, 0x7fffffff, 0x00020000);
    reg[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((long)gr * KB + kb) * 128 + c * 16), 0, 16 /* sc1 */);
  }
}
__device__ __forceinline__ void store_tile_lds(unsigned char *dst, const u32x4 (&reg)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; i++) *reinterpret_cast<u32x4 *>(dst + (w * 4 + i) * 1024 + lane * 16) = reg[i];
}

__device__ __forceinline__ halfx8 frag(const unsigned char *tile, int row, int chunk) {
  return *reinterpret_cast<const halfx8 *>(tile + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

// Row tile of the i-th work slot in readiness order of a bidirectional
// producer: tile rt (frames t0..t1) is complete once direction 0 has reached
// t1 and direction 1 has reached T-1-t0, i.e. at step max(t1, T-1-t0): the
// middle of the sequence first, then alternately outwards.
__device__ __forceinline__ int stream_row_tile(int i, int nrt, int sT, int sN) {
  // ready step of tile rt: max(t1(rt), T-1-t0(rt)); sort key, ties by rt.
  // Binary-search-free: walk outwards from the middle tile.
  const int tmid = (sT - 1) / 2;
  const int mid = min(nrt - 1, (tmid * sN) / TB);
  // interleave mid, mid-1, mid+1, mid-2, ... (exact ordering of ready steps
  // is not required for correctness, only for overlap)
  const int L = mid, R = nrt - 1 - mid;  // tiles left / right of the middle one
  if (i > 2 * min(L, R)) return L < R ? mid + (i - L) : mid - (i - R);
  const int k = (i + 1) / 2;
  return (i & 1) ? mid - k : mid + k;
}

// ---- waits on other workgroups ------------------------------------------
// All polling is done by wave 0 with every lane active and every exit
// decision made wave-uniform (readfirstlane), and the waves choose between
// polling and waiting on the barrier by a scalar branch on their wave index.
// (Thread-0 spin loops followed by a barrier let the compiler structure the
// barrier into exec-masked control flow: waves 1-3 then ran on without wave
// 0, observed as a hang on the GPU.)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o));
  return __builtin_amdgcn_readfirstlane(v);
}

// wave-level: true once every flag word f[32 g], g < nwg, holds >= need
// (false after a timeout or another party's error; then err bit 2 is set)
__device__ __forceinline__ unsigned wave_flags_min(const unsigned *f, int nwg) {
  unsigned m = 0xffffffffu;
  for (int g = threadIdx.x & 63; g < nwg; g += 64)
    m = min(m, __hip_atomic_load(f + 32L * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return wave_min_u32(m);
}
// A wait that runs out of time itself (no error posted yet) also sets bit
// 8 + site of err: which wait it was (0 producer rows, 1 pack jobs / tile
// arrivals, 2 pinned-XCD registrations, 3 producer epochs) -- the other
// bits are set by whoever saw the error first.
__device__ __forceinline__ bool wave_timed_out(unsigned *err, int spins, unsigned long long t0, int site) {
  if ((spins & 255) != 255) return false;
  const unsigned e = err ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT)) : 0u;
  if (e != 0u) return true;
  const bool late = __builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks;
  if (late && err && (threadIdx.x & 63) == 0) atomicOr(err, 0x100u << site);
  return late;
}
__device__ __forceinline__ void wave_fail(unsigned *err) {
  if ((threadIdx.x & 63) == 0 && err) atomicOr(err, 2u);
}

// Waiting for a producer that is `gap` steps (~3 us each) short: sleep for
// gap - 1 steps instead of re-polling its flag lines every ~0.2 us -- up to
// 176 blocks poll the same lines the recurrence itself polls and stores
__device__ __forceinline__ void backoff(int gap) {
  if (gap > 2) {
    const int n = min(gap - 1, 64);
    for (int i = 0; i < n; i++) __builtin_amdgcn_s_sleep(80);  // 80 x 64 clocks: ~2.4 us at 2.1 GHz
  } else {
    __builtin_amdgcn_s_sleep(8);
  }
}

// (Inside the polling loops every branch is wave-uniform; the single-lane
// stores of the outcome come after the loop: a lane-0 store in front of a
// `break` let the compiler leave lane 0 of wave 0 switched off, observed as
// EXEC = ...fffe and a workgroup running on without its thread 0.)
__device__ void x3p_wait_rows(const PParams &p, int m0, int *prog, int pd) {
  // prog[0..1]: steps known published by directions 0 / 1 (LDS cache; every
  // wave reads it before the barrier, wave 0 writes it only after).
  // pd = 0 / 1: only that producer direction's rows are needed (-1: both)
  const int r1 = min(p.M, m0 + TB) - 1;
  const int t0 = m0 / p.sN, t1 = r1 / p.sN;
  const int need0 = pd == 1 ? -1 : t1, need1 = pd == 0 ? -1 : p.sT - 1 - t0;
  const bool ok = __builtin_amdgcn_readfirstlane(prog[0] >= need0 && prog[1] >= need1);
  __syncthreads();
  if (ok) return;
  if (wave_id() == 0) {
    const unsigned long long ts = __builtin_amdgcn_s_memrealtime();
    int s0 = 0, s1 = 0, spins = 0;
    bool failed = false;
    while (true) {
      // epochs: step + 2; the slowest row group decides ([group][dir][wg] lines)
      s0 = s1 = 1 << 30;
      for (int gi = 0; gi < p.srg; gi++) {
        s0 = min(s0, (int)wave_flags_min(p.sflags + 32L * (2 * gi) * p.snwg, p.snwg) - 2);
        s1 = min(s1, (int)wave_flags_min(p.sflags + 32L * (2 * gi + 1) * p.snwg, p.snwg) - 2);
      }
      if (s0 >= need0 && s1 >= need1) break;
      failed = wave_timed_out(p.serr, spins++, ts, 0);
      if (failed) break;  // the producer stopped: flag it, finish on whatever is there
      backoff(p.backoff ? max(need0 - s0, need1 - s1) : 0);
    }
    if (failed) s0 = s1 = 1 << 30;
    if (threadIdx.x == 0) { prog[0] = s0; prog[1] = s1; }
    if (failed) wave_fail(p.serr);
  }
  __syncthreads();
}

// ---- backward stream helpers -------------------------------------------
// wave 0 waits for a device counter to reach v, then the workgroup barrier
__device__ __forceinline__ void wait_count(const int *a, int v, unsigned *err) {
  if (wave_id() == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool failed = false;
    int i = 0;
    while (true) {
      const int x = __builtin_amdgcn_readfirstlane(__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (x >= v) break;
      failed = wave_timed_out(err, i++, t0, 1);
      if (failed) break;
      __builtin_amdgcn_s_sleep(4);
    }
    if (failed) wave_fail(err);
  }
  __syncthreads();
}

// true when this block runs on an XCD that an XCD-pinned producer occupies
// (block-uniform): wave 0 waits until the producer's workgroups registered
// p.xcd_count XCDs in *p.xcd_word (bounded, as the other waits), then looks
// up its own.  Such blocks leave before taking work -- spinning on the
// producer's flags there they would keep its workgroups off their CUs.
__device__ bool on_pinned_xcd(const PParams &p, int *bc) {
  if (!p.xcd_word) return false;
  if (wave_id() == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned m = 0;
    bool failed = false;
    int i = 0;
    while (true) {
      m = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p.xcd_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (__builtin_popcount(m) >= p.xcd_count) break;
      failed = wave_timed_out(p.serr, i++, t0, 2);
      if (failed) break;
      __builtin_amdgcn_s_sleep(4);
    }
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) *bc = failed ? 1 : (int)((m >> (x & 0xfu)) & 1u);
    if (failed) wave_fail(p.serr);
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*bc) != 0;
}

// wait until every workgroup of producer direction d has published epoch
// >= need (seen[d]: the last minimum seen, LDS)
__device__ void wait_epoch(const PParams &p, int d, int need, int *seen) {
  const bool ok = __builtin_amdgcn_readfirstlane(seen[d] >= need);
  __syncthreads();
  if (ok) return;
  if (wave_id() == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool failed = false;
    int m = 0, spins = 0;
    while (true) {
      m = 1 << 30;
      for (int gi = 0; gi < p.srg; gi++)
        m = min(m, (int)wave_flags_min(p.sflags + 32L * (2 * gi + d) * p.snwg, p.snwg));
      if (m >= need) break;
      failed = wave_timed_out(p.serr, spins++, t0, 3);
      if (failed) break;
      backoff(p.backoff ? need - m : 0);
    }
    if (threadIdx.x == 0) seen[d] = failed ? 1 << 30 : m;
    if (failed) wave_fail(p.serr);
  }
  __syncthreads();
}

// the two directions' partial products of output tile (tm, tn) meet here:
// the first to arrive publishes its partial (sc1), the second adds it and
// writes C.  dx = part0 + part1 either way (fp addition commutes), so the
// result does not depend on the order of arrival.
__device__ __forceinline__ void bwd_combine(const PParams &p, floatx4 (&acc)[4][4], const int (&ea)[4][4], const int (&eb)[4],
                            int tm, int tn, int m0, int n0, int wm, int wn, int fr, int fq, int *bc) {
  int *arr = p.arrive + (long)tm * p.gx + tn;
  if (threadIdx.x == 0) *bc = __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool first = __builtin_amdgcn_readfirstlane(*bc) == 0;
  const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.part, 0, 0x7fffffff, 0x00020000);
  if (!first) wait_count(arr, 4, p.serr);
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int col = n0 + wn + j * 16 + fr;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + wm + i * 16 + fq * 4 + r;
        if (row >= p.M) continue;
        const float v = ldexpf(acc[i][j][r], -(ea[i][r] + eb[j]));
        const int off = (int)(((long)row * p.N + col) * 4);
        if (first) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rp, off, 0, 16);
        } else {
          const float o = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, off, 0, 16));
          p.C[(long)row * p.ldc + col] = v + o;
        }
      }
    }
  // unconditional barrier (see fwd_combine)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (first && threadIdx.x == 0) __hip_atomic_fetch_add(arr, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Direction-split streaming (p.sdir): the K of the projection is [h_fwd |
// h_bwd], and the forward half of frame t is ready at producer step t, the
// backward half at step T-1-t -- so each C tile is two half-K jobs, taken in
// the order their rows appear (forward half: row tiles ascending, backward
// half: descending), and the work is spread over the whole recurrence instead
// of its second half.  The halves meet in C: the first to arrive stores its
// partial (sc1), the second adds it, its own and the bias and writes C.
// (v0 + v1) + bias is the same either way round, so C does not depend on the
// order of arrival.
__device__ __forceinline__ void fwd_combine(const PParams &p, floatx4 (&acc)[4][4], const int (&ea)[4][4],
                                            const int (&eb)[4], int tm, int tn, int b, int m0, int n0, int wm, int wn,
                                            int fr, int fq, int *bc) {
  const long tile = ((long)tm * p.batch + b) * p.gx + tn;
  int *arr = p.arrive + tile;
  if (threadIdx.x == 0) *bc = __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool first = __builtin_amdgcn_readfirstlane(*bc) == 0;
  // the partial travels in the accumulator layout: thread t's (i, j) fragment
  // is 16 B at [tile][i * 4 + j][t], so both halves store / load whole,
  // coalesced 16-B chunks (sc1: the other half may run on another XCD)
  const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.part + tile * (TB * TB), 0, TB * TB * 4, 0x00020000);
  floatx4 v[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int r = 0; r < 4; r++) v[i][j][r] = ldexpf(acc[i][j][r], -(ea[i][r] + eb[j]));
  if (first) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[i][j]), rp,
                                               ((i * 4 + j) * NTH + (int)threadIdx.x) * 16, 0, 16);
  } else {
    if (!(p.dbg & 1)) wait_count(arr, 4, p.serr);
    float *C = p.C + (long)b * p.sC;
    const float *bias = p.bias ? p.bias + (long)b * p.sBias : nullptr;
    const float *bias2 = p.bias2 ? p.bias2 + (long)b * p.sBias : nullptr;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const floatx4 o = __builtin_bit_cast(
            floatx4, __builtin_amdgcn_raw_buffer_load_b128(rp, ((i * 4 + j) * NTH + (int)threadIdx.x) * 16, 0, 16));
        const int col = n0 + wn + j * 16 + fr;
        if (col >= p.N) continue;
        float badd = 0.f;
        if (bias) badd += bias[col];
        if (bias2) badd += bias2[col];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = m0 + wm + i * 16 + fq * 4 + r;
          if (row < p.M) C[(long)row * p.ldc + col] = (v[i][j][r] + o[r]) + badd;
        }
      }
  }
  // the barrier is unconditional: under `if (first)` (as bwd_combine had it)
  // the compiler let waves of this inlined copy skip it (observed: a hang)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (first && threadIdx.x == 0) __hip_atomic_fetch_add(arr, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SM (source mode): 0 packed A via LDS-DMA; 1 A = a forward producer's
// exchange images (sc1 register loads); 2 packed A just written by other CUs
// (LDS-DMA with sc1, exponents read with sc1) and the two-direction combine
// epilogue of the backward stream.
// BFM: the operands are bf16-packed ([row][KB][64] bf16, 64 consecutive k per
// 128-B block): a stage is two v_mfma_f32_16x16x32_bf16 (chunks fq and 4 + fq)
// instead of the three split-fp16 products, no exponents.
// one k block of MFMAs on the LDS stage `cur` (A and B tiles)
template <bool BFM>
__device__ __forceinline__ void x3p_kblock(const unsigned char *cur, int wm, int wn, int fr, int fq,
                                           floatx4 (&acc)[4][4]) {
  halfx8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    ah[i] = frag(cur, wm + i * 16 + fr, fq);
    al[i] = frag(cur, wm + i * 16 + fr, 4 + fq);
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    bh[j] = frag(cur + TILEB, wn + j * 16 + fr, fq);
    bl[j] = frag(cur + TILEB, wn + j * 16 + fr, 4 + fq);
  }
  if constexpr (BFM) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah[i]),
                                                            __builtin_bit_cast(bf16x8, bh[j]), acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al[i]),
                                                            __builtin_bit_cast(bf16x8, bl[j]), acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
  }
}

// k loop of the register-loaded A modes (SM 1: a forward producer's images,
// SM 2: rows packed by other workgroups; both sc1 loads whose latency is a
// MALL / other-XCD round trip): A is prefetched TWO k blocks ahead in a
// two-slot register ring (the loop is unrolled by two so the ring indices are
// static), B by LDS-DMA one block ahead, and the stage hand-over waits with a
// counted vmcnt that leaves the newest A prefetch in flight plus a raw
// s_barrier (a __syncthreads() would drain it).  Issue order per block it:
// B(it + 1) then A(it + 2), so vmcnt(4) at the end of block it means B(it + 1)
// and A(it + 1) have landed.  The body is straight-line (the loads past the
// last block re-read it, clamped, and are drained after the loop): with the
// loads under branches the compiler put a vmcnt(0) in front of every
// prefetch.  Even block counts only (the caller falls back otherwise).
template <int SM, bool BFM>
__device__ __forceinline__ void x3p_kloop_reg(const PParams &p, unsigned char *lds, const _Float16 *A,
                                              const _Float16 *B, int m0, int n0, int kb0, int nk, int wm, int wn,
                                              int fr, int fq, floatx4 (&acc)[4][4]) {
  u32x4 r0[4], r1[4];
  const int kbl = kb0 + nk - 1;
  auto loadA = [&](int kb, u32x4 (&r)[4]) {
    if constexpr (SM == 1) load_tile_xch(p, A, m0, min(kb, kbl), r);
    else load_tile_sc1(A, p.M, m0, p.KB, min(kb, kbl), r);
  };
  auto stage_wait = [&]() {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  loadA(kb0, r0);
  issue_tile(B, p.N, n0, p.KB, kb0, lds + TILEB);
  loadA(kb0 + 1, r1);
  store_tile_lds(lds, r0);
  stage_wait();
  // block it: cur holds A(it), B(it); rn holds A(it + 1); rf is free
  auto body = [&](int it, u32x4 (&rf)[4], u32x4 (&rn)[4]) {
    unsigned char *cur = lds + (it & 1) * 2 * TILEB;
    unsigned char *nxt = lds + ((it + 1) & 1) * 2 * TILEB;
    issue_tile(B, p.N, n0, p.KB, min(kb0 + it + 1, kbl), nxt + TILEB);
    loadA(kb0 + it + 2, rf);
    x3p_kblock<BFM>(cur, wm, wn, fr, fq, acc);
    store_tile_lds(nxt, rn);
    stage_wait();
  };
  for (int it = 0; it < nk; it += 2) {
    body(it, r0, r1);
    body(it + 1, r1, r0);
  }
  // the clamped loads past the last block land before anyone reuses the stages
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int SM, bool BFM = false>
__device__ __forceinline__ void x3p_tile(const PParams &p, unsigned char *lds, int tm, int tn, int b, int ks, int *prog) {
  constexpr bool STREAM = SM == 1;
  const _Float16 *A = p.A + (long)b * p.sA;
  const _Float16 *B = p.B + (long)b * p.sB;
  const int m0 = tm * TB, n0 = tn * TB;
  const int kb0 = ks * p.kbchunk, kb1 = min(p.KB, kb0 + p.kbchunk);
  const int nk = kb1 > kb0 ? kb1 - kb0 : 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int fr = lane & 15, fq = lane >> 4;

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (STREAM) x3p_wait_rows(p, m0, prog, p.sdir && !(p.dbg & 2) ? ks : -1);
  if constexpr (SM != 0) {
    if (!(p.dbg & 32) && nk >= 2 && !(nk & 1)) {
      x3p_kloop_reg<SM, BFM>(p, lds, A, B, m0, n0, kb0, nk, wm, wn, fr, fq, acc);
      goto epilogue;
    }
  }
  {
  // LDS: [2 stages][A tile | B tile]
  u32x4 ra[4];
  if (nk > 0) {
    if (STREAM) {
      load_tile_xch(p, A, m0, kb0, ra);
      store_tile_lds(lds, ra);
    } else if (SM == 2) {  // rows packed by other workgroups: sc1 loads to registers (not LDS-DMA)
      load_tile_sc1(A, p.M, m0, p.KB, kb0, ra);
      store_tile_lds(lds, ra);
    } else {
      issue_tile(A, p.M, m0, p.KB, kb0, lds);
    }
    issue_tile(B, p.N, n0, p.KB, kb0, lds + TILEB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; it++) {
    unsigned char *cur = lds + (it & 1) * 2 * TILEB;
    unsigned char *nxt = lds + ((it + 1) & 1) * 2 * TILEB;
    if (it + 1 < nk) {
      if (STREAM) load_tile_xch(p, A, m0, kb0 + it + 1, ra);
      else if (SM == 2) load_tile_sc1(A, p.M, m0, p.KB, kb0 + it + 1, ra);
      else issue_tile(A, p.M, m0, p.KB, kb0 + it + 1, nxt);
      issue_tile(B, p.N, n0, p.KB, kb0 + it + 1, nxt + TILEB);
    }
    halfx8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      ah[i] = frag(cur, wm + i * 16 + fr, fq);
      al[i] = frag(cur, wm + i * 16 + fr, 4 + fq);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      bh[j] = frag(cur + TILEB, wn + j * 16 + fr, fq);
      bl[j] = frag(cur + TILEB, wn + j * 16 + fr, 4 + fq);
    }
    if constexpr (BFM) {
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah[i]),
                                                              __builtin_bit_cast(bf16x8, bh[j]), acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al[i]),
                                                              __builtin_bit_cast(bf16x8, bl[j]), acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
    }
    if ((STREAM || SM == 2) && it + 1 < nk) store_tile_lds(nxt, ra);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  }
epilogue:

  // epilogue: acc[i][j][r] -> C[m0+wm+16i+4fq+r][n0+wn+16j+fr], times 2^-(eA + eB)
  const int *eA = p.eA ? p.eA + (long)b * p.seA : nullptr;
  const int *eB = p.eB ? p.eB + (long)b * p.seB : nullptr;
  int eb[4], ea[4][4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int col = n0 + wn + j * 16 + fr;
    eb[j] = col < p.N ? (p.eB ? eB[col] : p.eB0) : 0;
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = m0 + wm + i * 16 + fq * 4 + r;
      ea[i][r] = row >= p.M || BFM ? 0
                 : SM == 2  ? __hip_atomic_load(eA + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : p.eA     ? eA[row]
                            : p.eA0;
    }
  if (SM == 2) {
    bwd_combine(p, acc, ea, eb, tm, tn, m0, n0, wm, wn, fr, fq, prog);
    return;
  }
  if (STREAM && p.sdir && !(p.dbg & 4)) {
    fwd_combine(p, acc, ea, eb, tm, tn, b, m0, n0, wm, wn, fr, fq, prog + 2);
    return;
  }
  if (p.split > 1) {
    float *W = p.ws + ((long)ks * p.batch + b) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int col = n0 + wn + j * 16 + fr;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = m0 + wm + i * 16 + fq * 4 + r;
          if (row < p.M) W[(long)row * p.N + col] = ldexpf(acc[i][j][r], -(ea[i][r] + eb[j]));
        }
      }
    return;
  }
  float *C = p.C + (long)b * p.sC;
  const float *bias = p.bias ? p.bias + (long)b * p.sBias : nullptr;
  const float *bias2 = p.bias2 ? p.bias2 + (long)b * p.sBias : nullptr;
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int col = n0 + wn + j * 16 + fr;
      if (col >= p.N) continue;
      float badd = 0.f;
      if (bias) badd += bias[col];
      if (bias2) badd += bias2[col];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + wm + i * 16 + fq * 4 + r;
        if (row < p.M) {
          float *c = C + (long)row * p.ldc + col;
          float v = p.alpha * ldexpf(acc[i][j][r], -(ea[i][r] + eb[j])) + badd;
          if (p.beta != 0.f) v += p.beta * *c;
          *c = v;
        }
      }
    }
}

constexpr size_t kLdsBase = 2 * 2 * TILEB + 16, kLdsStream = 96 * 1024;
__host__ __device__ inline int stream_total(const PParams &p) { return p.nrt * p.batch * p.gx * (p.sdir ? 2 : 1); }

__device__ __forceinline__ void decode_tile(const PParams &p, int id, int total, bool remap, int &tm, int &tn,
                                            int &b, int &ks) {
  const int q = total >> 3, rr = total & 7, xcd = id & 7, loc = id >> 3;
  const int wl = remap ? (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc : id;
  const int bz = wl / p.tiles, wg = wl - bz * p.tiles;
  if (remap) {
    // groups of 8 tile rows, column by column inside a group: the 32 blocks
    // an XCD runs at once cover 8 row x 4 column tiles (12 panels of A and B
    // in its L2) instead of one row of tiles (1 + gx panels); 8192^3 bf16
    // 0.42 -> 0.45 of peak, the train step's shapes unchanged (±1 %)
    const int rows = p.tiles / p.gx, per = 8 * p.gx;
    const int grp = wg / per, first = grp * 8, w = wg - grp * per;
    const int gsz = min(8, rows - first);
    tm = first + w % gsz; tn = w / gsz;
  } else {
    tn = wg % p.gx; tm = wg / p.gx;
  }
  b = bz % p.batch; ks = bz / p.batch;
}

template <bool STREAM, bool BFM = false>
__global__ __launch_bounds__(NTH, 2) void gemm_x3p_kernel(PParams p) {
  // ONE shared array (a second __shared__ object can make hipcc wait vmcnt(0)
  // before LDS reads while a DMA is in flight); streaming launches ask for
  // 96 KB so that no block shares a CU with a producer workgroup
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB);
  int *prog = next + 1;
  const int total = STREAM ? stream_total(p) : p.tiles * p.batch * p.split;
  if (STREAM && threadIdx.x == 0) { prog[0] = -1; prog[1] = -1; }
  if (STREAM && on_pinned_xcd(p, prog + 2)) return;  // before taking any job
  if (p.counter) {
    while (true) {
      if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
      __syncthreads();
      const int id = __builtin_amdgcn_readfirstlane(*next);
      __syncthreads();
      if (id >= total) break;
      int tm, tn, b, ks;
      if (STREAM) {  // id = (row slot * batch + b) * gx + tn; no split-K
        tn = id % p.gx;
        const int rest = id / p.gx;
        b = rest % p.batch;
        const int slot = rest / p.batch;
        if (p.sdir) {  // slot = 2 j + producer direction: its K half of row tile j (dir 0) / nrt-1-j (dir 1)
          const int pd = slot & 1, j = slot >> 1;
          x3p_tile<1, BFM>(p, lds, pd == 0 ? j : p.nrt - 1 - j, tn, b, pd, prog);
        } else {
          tm = stream_row_tile(slot, p.nrt, p.sT, p.sN);
          x3p_tile<1, BFM>(p, lds, tm, tn, b, 0, prog);
        }
      } else {
        decode_tile(p, id, total, false, tm, tn, b, ks);
        x3p_tile<0, BFM>(p, lds, tm, tn, b, ks, prog);
      }
    }
    return;
  }
  if (!STREAM) {
    for (int id = blockIdx.x; id < total; id += gridDim.x) {
      int tm, tn, b, ks;
      decode_tile(p, id, total, true, tm, tn, b, ks);
      x3p_tile<0, BFM>(p, lds, tm, tn, b, ks, prog);
    }
  }
}

// ---- 256 x 256 tiles for the large GEMMs ----------------------------------
// Same packed operands and swizzled 128-B row images as x3p_tile, at 4x the
// tile area: 512 threads = 8 waves as 2 (M) x 4 (N), each wave a 128 x 64
// block of C (8 x 4 accumulators).  Per stage (one 128-B k block of both
// operands, 64 KB) a wave issues 96 split-fp16 (or 64 bf16) MFMAs against 24
// fragment reads, so the stage's LDS-DMA of the next block (8 x 16 B per
// thread) lands behind ~3000 SIMD cycles of matrix work; two stages (128 KB
// LDS), one workgroup per CU, one barrier per stage.  Tile ids are dealt to
// the XCDs in contiguous runs (decode_tile's remap) so that the blocks of an
// XCD share A and B panels in its L2.
constexpr int TB2 = 256, NTH2 = 512, TILEB2 = TB2 * ROWB;  // 32 KB per operand tile per stage
constexpr size_t kLds256 = 2 * 2 * (size_t)TILEB2 + 16;

__device__ __forceinline__ void issue_tile256(const _Float16 *__restrict__ P, int rows, int r0, int KB, int kb,
                                              unsigned char *dst) {
  // wave w fills rows [32 w, 32 w + 32): 4 instructions of 8 rows x 128 B
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int q = w * 4 + i;
    const int r = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int gr = r0 + r;
    gr = gr < rows ? gr : rows - 1;  // rows past the edge: any valid row (results discarded)
    __builtin_amdgcn_global_load_lds(P + ((long)gr * KB + kb) * 64 + c * 8, dst + q * 1024, 16, 0, 0);
  }
}

// one row block (16 rows of the wave's 128) of a k block: 4 (bf16: 2 x 4)
// or 12 (split-fp16) MFMAs against the wave's B fragments.  TR: operands
// swapped, the accumulators hold C^T (lane (fr, fq): row fr, columns
// 4 fq .. 4 fq + 3 of the 16 x 16 block -- 16-B row pieces for the epilogue)
template <bool BFM, bool TR = false>
__device__ __forceinline__ void p256_row(floatx4 (&acc)[4], halfx8 ah, halfx8 al, const halfx8 (&bh)[4],
                                         const halfx8 (&bl)[4]) {
  auto mm = [](halfx8 a, halfx8 b, floatx4 c) {
    if constexpr (BFM) {
      return TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b), __builtin_bit_cast(bf16x8, a),
                                                          c, 0, 0, 0)
                : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                          c, 0, 0, 0);
    } else {
      return TR ? __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c, 0, 0, 0)
                : __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
  };
  if constexpr (BFM) {
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = mm(ah, bh[j], acc[j]);
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = mm(al, bl[j], acc[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = mm(ah, bh[j], acc[j]);
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = mm(ah, bl[j], acc[j]);
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = mm(al, bh[j], acc[j]);
  }
}

// k loop with the next stage's LDS-DMA spread over the MFMAs: the wave's 8
// pieces (4 of A, 4 of B) are issued two per row block over the first four of
// its eight row blocks, between the MFMAs,
// instead of as one block of address arithmetic + m0 writes at the top of the
// iteration (where both waves of a SIMD issued them at once, right after the
// barrier, with no matrix work to hide behind).  Source pointers are computed
// once per tile; the loads of the last iteration re-read the last k block
// (clamped) so the body is straight-line.
// AUXA: cache policy of the A pieces (16: sc1, rows packed by other CUs
// while this kernel runs)
template <bool BFM, int AUXA = 0, bool TR = false>
__device__ __forceinline__ void p256_kloop_spread(const _Float16 *A, const _Float16 *B, int M, int N, int KB, int m0,
                                                  int n0, int kb0, int nk, unsigned char *lds, int wm, int wn, int fr,
                                                  int fq, floatx4 (&acc)[8][4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const _Float16 *src[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int q = w * 4 + (i & 3);
    const int r = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = i < 4 ? min(m0 + r, M - 1) : min(n0 + r, N - 1);
    src[i] = (i < 4 ? A : B) + ((long)gr * KB + kb0) * 64 + c * 8;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (i < 4) __builtin_amdgcn_global_load_lds(src[i], lds + (w * 4 + i) * 1024, 16, 0, AUXA);
    else __builtin_amdgcn_global_load_lds(src[i], lds + TILEB2 + (w * 4 + (i & 3)) * 1024, 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; it++) {
    unsigned char *cur = lds + (it & 1) * 2 * TILEB2;
    unsigned char *nxt = lds + ((it + 1) & 1) * 2 * TILEB2;
    const long adv = (long)min(it + 1, nk - 1) * 64;
    halfx8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      bh[j] = frag(cur + TILEB2, wn + j * 16 + fr, fq);
      bl[j] = frag(cur + TILEB2, wn + j * 16 + fr, 4 + fq);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (i < 4) {  // two pieces per row block of the first half: the last lands behind half the MFMAs
#pragma unroll
        for (int h = 2 * i; h < 2 * i + 2; h++) {
          if (h < 4) __builtin_amdgcn_global_load_lds(src[h] + adv, nxt + (w * 4 + h) * 1024, 16, 0, AUXA);
          else __builtin_amdgcn_global_load_lds(src[h] + adv, nxt + TILEB2 + (w * 4 + (h & 3)) * 1024, 16, 0, 0);
        }
      }
      const halfx8 ah = frag(cur, wm + i * 16 + fr, fq);
      const halfx8 al = frag(cur, wm + i * 16 + fr, 4 + fq);
      p256_row<BFM, TR>(acc[i], ah, al, bh, bl);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

template <bool BFM>
__device__ __forceinline__ void p256_tile(const PParams &p, unsigned char *lds, int tm, int tn, int b, int ks) {
  const _Float16 *A = p.A + (long)b * p.sA;
  const _Float16 *B = p.B + (long)b * p.sB;
  const int m0 = tm * TB2, n0 = tn * TB2;
  const int kb0 = ks * p.kbchunk, kb1 = min(p.KB, kb0 + p.kbchunk);
  const int nk = kb1 > kb0 ? kb1 - kb0 : 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 2) * 128, wn = (wid & 3) * 64;
  const int fr = lane & 15, fq = lane >> 4;
  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // default: the spread loop for split-fp16 (measured +4..10 %: dW 0.476 ->
  // 0.50-0.52, 8192^3 0.527 -> 0.555 of the f16 issue rate), the block loop
  // for bf16 (equal or 1-3 % faster there: fewer MFMAs per stage to hide the
  // DMA issue behind)
  if (p.p256v == 2 || (p.p256v == 0 && !BFM)) {
    if (nk > 0) p256_kloop_spread<BFM, 0, true>(A, B, p.M, p.N, p.KB, m0, n0, kb0, nk, lds, wm, wn, fr, fq, acc);
  } else {
  if (nk > 0) {
    issue_tile256(A, p.M, m0, p.KB, kb0, lds);
    issue_tile256(B, p.N, n0, p.KB, kb0, lds + TILEB2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; it++) {
    unsigned char *cur = lds + (it & 1) * 2 * TILEB2;
    unsigned char *nxt = lds + ((it + 1) & 1) * 2 * TILEB2;
    if (it + 1 < nk) {
      issue_tile256(A, p.M, m0, p.KB, kb0 + it + 1, nxt);
      issue_tile256(B, p.N, n0, p.KB, kb0 + it + 1, nxt + TILEB2);
    }
    halfx8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      bh[j] = frag(cur + TILEB2, wn + j * 16 + fr, fq);
      bl[j] = frag(cur + TILEB2, wn + j * 16 + fr, 4 + fq);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const halfx8 ah = frag(cur, wm + i * 16 + fr, fq);
      const halfx8 al = frag(cur, wm + i * 16 + fr, 4 + fq);
      p256_row<BFM, true>(acc[i], ah, al, bh, bl);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  }
  // epilogue, transposed accumulators: acc[i][j][c] -> C[m0+wm+16i+fr][n0+wn+16j+4fq+c],
  // times 2^-(eA + eB); one 16-B store per (i, j) where the row piece is aligned
  const int *eA = p.eA ? p.eA + (long)b * p.seA : nullptr;
  const int *eB = p.eB ? p.eB + (long)b * p.seB : nullptr;
  float *W = p.split > 1 ? p.ws + ((long)ks * p.batch + b) * (long)p.M * p.N : nullptr;
  float *C = p.C + (long)b * p.sC;
  const float *bias = p.bias ? p.bias + (long)b * p.sBias : nullptr;
  const float *bias2 = p.bias2 ? p.bias2 + (long)b * p.sBias : nullptr;
  float *const O = W ? W : C;
  const long ldo = W ? p.N : p.ldc;
  const bool vec = ((reinterpret_cast<unsigned long>(O) & 15) == 0) && (ldo & 3) == 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int col0 = n0 + wn + j * 16 + fq * 4;
    int eb[4];
    float badd[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int col = col0 + c;
      eb[c] = col < p.N ? (eB ? eB[col] : p.eB0) : 0;
      badd[c] = 0.f;
      if (!W && col < p.N) {
        if (bias) badd[c] += bias[col];
        if (bias2) badd[c] += bias2[col];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int row = m0 + wm + i * 16 + fr;
      if (row >= p.M || col0 >= p.N) continue;
      const int ea = eA ? eA[row] : p.eA0;
      float *o = O + (long)row * ldo + col0;
      floatx4 v;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        v[c] = ldexpf(acc[i][j][c], -(ea + eb[c]));
        if (!W) v[c] = p.alpha * v[c] + badd[c];
      }
      if (vec && col0 + 3 < p.N) {
        if (!W && p.beta != 0.f) {
          const floatx4 old = *reinterpret_cast<const floatx4 *>(o);
#pragma unroll
          for (int c = 0; c < 4; c++) v[c] += p.beta * old[c];
        }
        *reinterpret_cast<floatx4 *>(o) = v;
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++) {
          if (col0 + c < p.N) {
            float x = v[c];
            if (!W && p.beta != 0.f) x += p.beta * o[c];
            o[c] = x;
          }
        }
      }
    }
  }
}

// beside a pinned recurrence (X3PArgs::avoid_word): true on one of its XCDs
// (block-uniform; the word only ever gains bits)
__device__ __forceinline__ bool avoid_here(const PParams &p, int *bc) {
  if (!p.avoid) return false;
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    const unsigned m = __hip_atomic_load(p.avoid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *bc = (int)((m >> (x & 0xfu)) & 1u) && __builtin_popcount(m) < p.nxcd;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*bc) != 0;
}

template <bool BFM>
__global__ __launch_bounds__(NTH2, 1) void gemm_p256_kernel(PParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // ONE shared array
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB2);
  const int total = p.tiles * p.batch * p.split;
  if (avoid_here(p, next + 1)) return;
  if (p.counter) {  // dynamic scheduling (beside a persistent kernel)
    while (true) {
      if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
      __syncthreads();
      const int id = __builtin_amdgcn_readfirstlane(*next);
      __syncthreads();
      if (id >= total) break;
      int tm, tn, b, ks;
      decode_tile(p, id, total, false, tm, tn, b, ks);
      p256_tile<BFM>(p, lds, tm, tn, b, ks);
    }
    return;
  }
  for (int id = blockIdx.x; id < total; id += gridDim.x) {
    int tm, tn, b, ks;
    decode_tile(p, id, total, true, tm, tn, b, ks);
    p256_tile<BFM>(p, lds, tm, tn, b, ks);
  }
}

// two problems, one job space (p's jobs, then q's), p's tile counter
template <bool BFM>
__global__ __launch_bounds__(NTH2, 1) void gemm_p256_pair_kernel(PParams p, PParams q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // ONE shared array
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB2);
  const int t1 = p.tiles * p.batch * p.split, t2 = q.tiles * q.batch * q.split;
  if (avoid_here(p, next + 1)) return;
  while (true) {
    if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
    __syncthreads();
    const int id = __builtin_amdgcn_readfirstlane(*next);
    __syncthreads();
    if (id >= t1 + t2) break;
    int tm, tn, b, ks;
    if (id < t1) {
      decode_tile(p, id, t1, false, tm, tn, b, ks);
      p256_tile<BFM>(p, lds, tm, tn, b, ks);
    } else {
      decode_tile(q, id - t1, t2, false, tm, tn, b, ks);
      p256_tile<BFM>(q, lds, tm, tn, b, ks);
    }
  }
}

__global__ __launch_bounds__(256) void x3p_splitk_reduce(PParams p) {
  const long total = (long)p.batch * p.M * p.N;
  const long MN = (long)p.M * p.N;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int b = (int)(e / MN);
    const long rem = e - (long)b * MN;
    const int row = (int)(rem / p.N), col = (int)(rem - (long)row * p.N);
    float s = 0.f;
    for (int k = 0; k < p.split; k++) s += p.ws[((long)k * p.batch + b) * MN + rem];
    float *c = p.C + (long)b * p.sC + (long)row * p.ldc + col;
    float v = p.alpha * s;
    if (p.bias) v += p.bias[(long)b * p.sBias + col];
    if (p.bias2) v += p.bias2[(long)b * p.sBias + col];
    if (p.beta != 0.f) v += p.beta * *c;
    *c = v;
  }
}

__device__ __forceinline__ int split_exp_d(float mx) {
  int e = 0;
  (void)frexpf(mx, &e);
  return 14 - e;
}

__device__ __forceinline__ void split4(floatx4 v, int e, halfx4 &h, halfx4 &l) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const float x = ldexpf(v[j], e);
    h[j] = (_Float16)x;
    l[j] = (_Float16)(x - (float)h[j]);
  }
}

// Row packing: one wave per row; lane l holds k = 4 l + 256 i (i < KW), so a
// row of up to 256 KW values is read once.  bound > 0: fixed exponent.
template <int KW>
__global__ __launch_bounds__(256) void pack_rows_kernel(const float *__restrict__ X, long ldx, int R, int K, int KB,
                                                        long sX, _Float16 *__restrict__ out, long sOut,
                                                        int *__restrict__ eout, long sE, float bound, int vec) {
  const int b = blockIdx.y;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const float *x = X + (long)b * sX + (long)r * ldx;
  floatx4 v[KW];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < KW; i++) {
    const int k = 4 * lane + 256 * i;
    floatx4 t = {0.f, 0.f, 0.f, 0.f};
    if (vec && k + 3 < K) {
      t = *reinterpret_cast<const floatx4 *>(x + k);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) t[j] = k + j < K ? x[k + j] : 0.f;
    }
    v[i] = t;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(t[0]), fabsf(t[1])), fmaxf(fabsf(t[2]), fabsf(t[3]))));
  }
  int e;
  if (bound > 0.f) {
    e = split_exp_d(bound);
  } else {
    mx = wave_max_l63(mx);
    e = split_exp_d(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 63)));
  }
  _Float16 *o = out + (long)b * sOut + (long)r * KB * 64;
#pragma unroll
  for (int i = 0; i < KW; i++) {
    const int k = 4 * lane + 256 * i;
    if (k < KB * 32) {
      halfx4 h, l;
      split4(v[i], e, h, l);
      const int kb = k >> 5, off = k & 31;
      *reinterpret_cast<halfx4 *>(o + kb * 64 + off) = h;
      *reinterpret_cast<halfx4 *>(o + kb * 64 + 32 + off) = l;
    }
  }
  if (lane == 0 && eout) eout[(long)b * sE + r] = e;
}

// ---- backward stream: pack jobs + GEMM jobs in one persistent launch ----
// Rows of direction d of a backward recurrence's dGates (E) become available
// step by step (direction 0 from t = T-1 down, direction 1 from t = 0 up).
// Per (row tile, direction) slot: P pack jobs (rows -> packed hi/lo with a
// per-row exponent, sc1 stores, then done[d][rt] += 1) and gx GEMM jobs
// (wait done == P, then the tile with sc1 LDS-DMA, combine epilogue).  Slots
// alternate directions in production order; jobs are taken from one counter,
// so a GEMM job only ever waits for pack jobs that running blocks own.
template <int KW, bool BFM, int NWV = 4>
__device__ __forceinline__ void bwd_pack_rows(const PParams &p, int d, int r0, int r1) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int K = p.KB * (BFM ? 64 : 32);
  for (int r = r0 + w; r < r1; r += NWV) {
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p.E + (long)r * p.lde + d * p.edoff), 0,
                                                      K * 4, 0x00020000);
    floatx4 v[KW];
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < KW; i++) {
      const int k = 4 * lane + 256 * i;
      v[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (k < K) v[i] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rx, k * 4, 0, 16));
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[i][0]), fabsf(v[i][1])), fmaxf(fabsf(v[i][2]), fabsf(v[i][3]))));
    }
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(p.A) + (long)d * p.sA + (long)r * p.KB * 64, 0, p.KB * 128,
                                                      0x00020000);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    if constexpr (BFM) {  // bf16 rows [KB][64], no exponent
#pragma unroll
      for (int i = 0; i < KW; i++) {
        const int k = 4 * lane + 256 * i;
        if (k < K) {
          bf16x4 h;
#pragma unroll
          for (int j = 0; j < 4; j++) h[j] = (__bf16)v[i][j];
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), ro, k * 2, 0, 16);
        }
      }
      continue;
    }
    mx = wave_max_l63(mx);
    const int e = split_exp_d(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), 63)));
#pragma unroll
    for (int i = 0; i < KW; i++) {
      const int k = 4 * lane + 256 * i;
      if (k < K) {
        halfx4 h, l;
        split4(v[i], e, h, l);
        const int kb = k >> 5, off = k & 31;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), ro, (kb * 64 + off) * 2, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, l), ro, (kb * 64 + 32 + off) * 2, 0, 16);
      }
    }
    if (lane == 0)
      __hip_atomic_store(const_cast<int *>(p.eA) + (long)d * p.seA + r, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int KW, bool BFM>
__global__ __launch_bounds__(NTH, 2) void x3p_bwd_stream_kernel(PParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB);
  int *seen = next + 1;  // [2] producer epochs seen
  int *bc = next + 3;    // combine broadcast
  if (threadIdx.x == 0) { seen[0] = 0; seen[1] = 0; }
  const int J = p.P + p.gx, total = 2 * p.nrt * J, rows_per = TB / p.P;
  if (on_pinned_xcd(p, bc)) return;  // before taking any job
  while (true) {
    if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
    __syncthreads();
    const int id = __builtin_amdgcn_readfirstlane(*next);
    __syncthreads();
    if (id >= total) break;
    const int slot = id / J, r = id - slot * J, d = slot & 1, rank = slot >> 1;
    const int rt = d == 0 ? p.nrt - 1 - rank : rank;
    if (r < p.P) {
      const int ra = rt * TB + r * rows_per, rb = min(p.M, ra + rows_per);
      if (ra < rb) {
        // E rows of step s are stored one step later: complete at epoch s + 3
        // (s = steps done before it; the last step gets epoch T + 2 at exit)
        const int ta = ra / p.sN, tb = (rb - 1) / p.sN;
        wait_epoch(p, d, d == 0 ? p.sT + 2 - ta : tb + 3, seen);
        bwd_pack_rows<KW, BFM>(p, d, ra, rb);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(p.done + d * p.nrt + rt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // a barrier after the lane-0 atomic: with the atomic as the last thing
      // in the body hipcc structured the job loop as divergent (the loop latch
      // masks lanes off), which left lane 0 of wave 0 behind with the
      // barriers inside the loop still completing for the rest
      __syncthreads();
    } else {
      wait_count(p.done + d * p.nrt + rt, p.P, p.serr);
      x3p_tile<2, BFM>(p, lds, rt, r - p.P, d, 0, bc);
      __syncthreads();
    }
  }
}

// ---- the backward stream on 256 x 256 tiles ------------------------------
// x3p_bwd_stream_kernel's job list at the p256 tile (512 threads, 128 KB
// LDS, one block per CU): per (row tile, direction) slot P pack jobs of
// 256 / P rows (8 waves) and gx GEMM jobs of 256 x 256 over the direction's
// whole K, A by sc1 LDS-DMA (rows packed by other CUs during this launch).
// A 256 x 256 tile issues 2x the MFMAs per LDS byte of the 128 tile, so the
// dx GEMM keeps up with the recurrence on about a third of the CUs the 128
// version needed, and the rest run the weight GEMMs (gemm_x3p avoid_word).
// The two directions' partials meet in the accumulator layout
// (part + tile * 256 * 256: thread t's (i, j) fragment is 16 B at
// [i * 4 + j][t]): the first to arrive stores its partial (sc1), the second
// adds it and writes C -- part0 + part1 either way round.
// ks / S: this job's K-split of S (S > 1: a tail slot, its tile's partials
// meet in part2)
template <bool BFM>
__device__ __forceinline__ void p256_bwd_tile(const PParams &p, unsigned char *lds, int tm, int tn, int d, int *bc,
                                              int ks, int S) {
  const _Float16 *A = p.A + (long)d * p.sA, *B = p.B + (long)d * p.sB;
  const int m0 = tm * TB2, n0 = tn * TB2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 2) * 128, wn = (wid & 3) * 64;
  const int fr = lane & 15, fq = lane >> 4;
  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int kbs = (p.KB + S - 1) / S, kb0 = ks * kbs, nk = max(0, min(p.KB, kb0 + kbs) - kb0);
  // transposed accumulators (p256_row TR): lane (fr, fq) holds row
  // m0 + wm + 16 i + fr, columns n0 + wn + 16 j + 4 fq .. + 3 of C
  if (nk > 0) p256_kloop_spread<BFM, 16, true>(A, B, p.M, p.N, p.KB, m0, n0, kb0, nk, lds, wm, wn, fr, fq, acc);
  if constexpr (!BFM) {  // to values: 2^-(eA[row] + eB[col]) (eA written by other CUs: sc1 loads)
    const int *eA = p.eA + (long)d * p.seA, *eB = p.eB + (long)d * p.seB;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int eb[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int col = n0 + wn + j * 16 + fq * 4 + c;
        eb[c] = col < p.N ? eB[col] : 0;
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int row = m0 + wm + i * 16 + fr;
        const int ea = row < p.M ? __hip_atomic_load(eA + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#pragma unroll
        for (int c = 0; c < 4; c++) acc[i][j][c] = ldexpf(acc[i][j][c], -(ea + eb[c]));
      }
    }
  }
  // C row piece (i, j) of this lane: + bias + bias2 of each column (gemm_x3p's
  // order), one 16-B store where the piece is whole and aligned
  const bool vec = ((reinterpret_cast<unsigned long>(p.C) & 15) | (p.ldc & 3)) == 0;
  // the biases of this lane's 16 columns (a column's only: computed once)
  float bsum[4][4];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int col = min(n0 + wn + j * 16 + fq * 4 + c, p.N - 1);
        const long bo = (long)(col / p.bcols) * p.sBias + col % p.bcols;
        float badd = 0.f;
        badd += p.bias[bo];
        if (p.bias2) badd += p.bias2[bo];
        bsum[j][c] = badd;
      }
  }
  auto put = [&](int i, int j, floatx4 v) {
    const int row = m0 + wm + i * 16 + fr, col0 = n0 + wn + j * 16 + fq * 4;
    if (row >= p.M || col0 >= p.N) return;
    if (p.bias) {
#pragma unroll
      for (int c = 0; c < 4; c++) v[c] = v[c] + bsum[j][c];
    }
    float *o = p.C + (long)row * p.ldc + col0;
    if (vec && col0 + 3 < p.N) {
      *reinterpret_cast<floatx4 *>(o) = v;
    } else {
#pragma unroll
      for (int c = 0; c < 4; c++)
        if (col0 + c < p.N) o[c] = v[c];
    }
  };
  const long tile = (long)tm * p.gx + tn;
  int *arr = p.arrive + tile;
  // a tail tile (one of its directions split p.tails ways): every partial
  // goes to its slot q of [other direction's, split 0 .. tails - 1] in
  // part2, then arrives; the last arrival adds the slots up in q order (acc
  // is dead after the store: the tail costs the k loop no registers)
  const bool tail = p.tailr > 0 && (tm < p.tailr || tm >= p.nrt - p.tailr);
  if (tail) {
    const int n = p.tails + 1, q = S > 1 ? 1 + ks : 0;
    const int ti = tm < p.tailr ? tm : p.tailr + tm - (p.nrt - p.tailr);
    float *base = p.part2 + ((long)(ti * p.gx + tn) * n) * (TB2 * TB2);
    {
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(base + (long)q * (TB2 * TB2), 0, TB2 * TB2 * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rq,
                                                 ((i * 4 + j) * NTH2 + (int)threadIdx.x) * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) *bc = __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(*bc) == n - 1) {
      const auto rb = __builtin_amdgcn_make_buffer_rsrc(base, 0, n * TB2 * TB2 * 4, 0x00020000);
      for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) {
          const int off = ((i * 4 + j) * NTH2 + (int)threadIdx.x) * 16;
          floatx4 v = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 16));
          for (int qq = 1; qq < n; qq++)
            v += __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rb, off + qq * TB2 * TB2 * 4, 0, 16));
          put(i, j, v);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return;
  }
  if (threadIdx.x == 0) *bc = __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool first = __builtin_amdgcn_readfirstlane(*bc) == 0;
  const auto rp = __builtin_amdgcn_make_buffer_rsrc(p.part + tile * (TB2 * TB2), 0, TB2 * TB2 * 4, 0x00020000);
  if (first) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rp,
                                               ((i * 4 + j) * NTH2 + (int)threadIdx.x) * 16, 0, 16);
  } else {
    wait_count(arr, 4, p.serr);
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const floatx4 o = __builtin_bit_cast(
            floatx4, __builtin_amdgcn_raw_buffer_load_b128(rp, ((i * 4 + j) * NTH2 + (int)threadIdx.x) * 16, 0, 16));
        put(i, j, acc[i][j] + o);
      }
  }
  // unconditional barrier (see fwd_combine)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (first && threadIdx.x == 0) __hip_atomic_fetch_add(arr, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int KW, bool BFM>
__global__ __launch_bounds__(NTH2, 1) void x3p_bwd_stream256_kernel(PParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB2);
  int *seen = next + 1;  // [2] producer epochs seen
  int *bc = next + 3;    // combine broadcast
  if (threadIdx.x == 0) { seen[0] = 0; seen[1] = 0; }
  // slots of the regular ranks (P pack + gx GEMM jobs), then the tail ranks'
  // (P pack + gx x tails GEMM jobs)
  const int J0 = p.P + p.gx, J1 = p.P + p.gx * p.tails, nreg = 2 * (p.nrt - p.tailr);
  const int base1 = nreg * J0, total = base1 + 2 * p.tailr * J1, rows_per = TB2 / p.P;
  if (on_pinned_xcd(p, bc)) return;  // before taking any job
  while (true) {
    if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
    __syncthreads();
    const int id = __builtin_amdgcn_readfirstlane(*next);
    __syncthreads();
    if (id >= total) break;
    int slot, r;
    if (id < base1) {
      slot = id / J0;
      r = id - slot * J0;
    } else {
      slot = nreg + (id - base1) / J1;
      r = (id - base1) % J1;
    }
    const int d = slot & 1, rank = slot >> 1;
    // the producer's direction that walks the frames downwards takes the
    // row tiles from the last (a backward producer's direction 0, a forward
    // producer's direction 1)
    const bool down = (d == 0) != (p.fwdp != 0);
    const int rt = down ? p.nrt - 1 - rank : rank;
    if (r < p.P) {
      const int ra = rt * TB2 + r * rows_per, rb = min(p.M, ra + rows_per);
      if (ra < rb) {
        // E rows of step s are complete at epoch s + 3 (the last step's at T + 2)
        const int ta = ra / p.sN, tb = (rb - 1) / p.sN;
        wait_epoch(p, d, down ? p.sT + 2 - ta : tb + 3, seen);
        bwd_pack_rows<KW, BFM, NTH2 / 64>(p, d, ra, rb);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(p.done + d * p.nrt + rt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();  // (see x3p_bwd_stream_kernel: reconverge after the lane-0 atomic)
    } else {
      wait_count(p.done + d * p.nrt + rt, p.P, p.serr);
      const int S = rank >= p.nrt - p.tailr ? p.tails : 1, gj = r - p.P;
      p256_bwd_tile<BFM>(p, lds, rt, gj % p.gx, d, bc, gj / p.gx, S);
      __syncthreads();
    }
  }
}

// one item: 64 columns x KPI consecutive 32-k blocks (KPI = 4, 512
// contiguous bytes per packed row, measured slower: configs[1] dGates^T
// 351 -> 511 us, fewer blocks in flight)
constexpr int KPI = 1;
__device__ __forceinline__ void pack_cols_item(const float *__restrict__ X, long ldx, int R, int Cn, int KB, int shift,
                                               long sX, _Float16 *__restrict__ out, long sOut, int *__restrict__ eout,
                                               long sE, const unsigned *__restrict__ cmax, long sCm, float bound,
                                               int bx, int kq, int b, float (*tile)[65]) {
  const int c0 = bx * 64, kb0 = kq * KPI;
  const float *x = X + (long)b * sX;
  const int t = threadIdx.x;
  // load KPI * 32 rows x 64 columns (each row: 64 consecutive floats), 16 B
  // per lane where the rows are 16-B aligned (4 rows per wave instruction)
  if (((reinterpret_cast<unsigned long>(x) & 15) | (ldx & 3)) == 0) {
#pragma unroll
    for (int i = 0; i < 2 * KPI; i++) {
      const int kr = (t >> 4) + 16 * i, cc = (t & 15) * 4;
      const int k = kb0 * 32 + kr, src = k - shift;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (k < R && src >= 0 && src < R) {
        const float *xr = x + (long)src * ldx + c0 + cc;
        if (c0 + cc + 3 < Cn) {
          v = *reinterpret_cast<const floatx4 *>(xr);
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++) v[e] = c0 + cc + e < Cn ? xr[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; e++) tile[kr][cc + e] = v[e];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8 * KPI; i++) {
      const int kr = (t >> 6) + 4 * i, cc = t & 63;
      const int k = kb0 * 32 + kr, src = k - shift;
      float v = 0.f;
      if (k < R && src >= 0 && src < R && c0 + cc < Cn) v = x[(long)src * ldx + c0 + cc];
      tile[kr][cc] = v;
    }
  }
  __syncthreads();
  const int c = t >> 2, part = t & 3;
  if (c0 + c < Cn) {
    const int e = bound > 0.f ? split_exp_d(bound)
                              : split_exp_d(__uint_as_float(cmax[(long)b * sCm + c0 + c]));
    _Float16 *o = out + (long)b * sOut + ((long)(c0 + c) * KB + kb0) * 64;
#pragma unroll
    for (int q = 0; q < KPI; q++) {
      if (kb0 + q >= KB) break;
      halfx8 h, l;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const float xv = ldexpf(tile[q * 32 + part * 8 + j][c], e);
        h[j] = (_Float16)xv;
        l[j] = (_Float16)(xv - (float)h[j]);
      }
      *reinterpret_cast<halfx8 *>(o + q * 64 + part * 8) = h;
      *reinterpret_cast<halfx8 *>(o + q * 64 + 32 + part * 8) = l;
    }
    if (kb0 == 0 && part == 0 && eout) eout[(long)b * sE + c0 + c] = e;
  }
}

// Column packing (transpose): packed row c = column c of X, K = X's rows
// (k -> X row k - shift, zero outside [0, R)).  Exponent from cmax[c] (max |x|
// of the column, float bits) or the bound.  Item: 64 columns x KPI 32-k blocks
// (grid (columns / 64, KB / KPI, batch)).  With `avoid` (beside a pinned
// recurrence, X3PArgs::avoid_word) a 1-D grid takes runs of 8 items from
// a zeroed counter and the blocks on the recurrence's XCDs leave at once: a
// stream of short blocks cycling through its CUs kept the recurrence's
// workgroups from becoming resident for the length of the pack (configs[1]:
// ~230 us a layer).
__global__ __launch_bounds__(256) void pack_cols_kernel(const float *__restrict__ X, long ldx, int R, int Cn, int KB,
                                                        int shift, long sX, _Float16 *__restrict__ out, long sOut,
                                                        int *__restrict__ eout, long sE,
                                                        const unsigned *__restrict__ cmax, long sCm, float bound,
                                                        const unsigned *avoid, int nxcd, int batch, int *counter) {
  __shared__ float tile[32 * KPI][65];
  __shared__ int bc;
  if (!avoid) {
    pack_cols_item(X, ldx, R, Cn, KB, shift, sX, out, sOut, eout, sE, cmax, sCm, bound, blockIdx.x, blockIdx.y,
                   blockIdx.z, tile);
    return;
  }
  PParams q;
  q.avoid = avoid;
  q.nxcd = nxcd;
  if (avoid_here(q, &bc)) return;
  const int gx = (Cn + 63) / 64, KQ = (KB + KPI - 1) / KPI;
  const int items = gx * KQ * batch;
  while (true) {
    __syncthreads();  // bc and the tile are reused
    if (threadIdx.x == 0) bc = atomicAdd(counter, 8);
    __syncthreads();
    const int i0 = __builtin_amdgcn_readfirstlane(bc);
    if (i0 >= items) break;
    for (int it = i0; it < min(items, i0 + 8); it++) {
      const int bx = it % gx, r = it / gx;
      pack_cols_item(X, ldx, R, Cn, KB, shift, sX, out, sOut, eout, sE, cmax, sCm, bound, bx, r % KQ, r / KQ, tile);
      __syncthreads();
    }
  }
}

// bf16 packing: out[b][r][kb][64] = bf16(x[r][64 kb + j]), zero past K.
// Rows: one wave per row, lane l holds k = 4 l + 256 i.
template <int KW>
__global__ __launch_bounds__(256) void bf16_pack_rows_kernel(const float *__restrict__ X, long ldx, int R, int K,
                                                             int KB, long sX, __bf16 *__restrict__ out, long sOut,
                                                             int vec) {
  const int b = blockIdx.y;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const float *x = X + (long)b * sX + (long)r * ldx;
  __bf16 *o = out + (long)b * sOut + (long)r * KB * 64;
#pragma unroll
  for (int i = 0; i < KW; i++) {
    const int k = 4 * lane + 256 * i;
    if (k >= KB * 64) continue;
    floatx4 t = {0.f, 0.f, 0.f, 0.f};
    if (vec && k + 3 < K) {
      t = *reinterpret_cast<const floatx4 *>(x + k);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) t[j] = k + j < K ? x[k + j] : 0.f;
    }
    bf16x4 h;
#pragma unroll
    for (int j = 0; j < 4; j++) h[j] = (__bf16)t[j];
    *reinterpret_cast<bf16x4 *>(o + k) = h;
  }
}
// Columns (transpose): packed row c = column c of X over its R rows (row
// k - shift, zero outside).  Block: 64 columns x one 64-k block.
__global__ __launch_bounds__(256) void bf16_pack_cols_kernel(const float *__restrict__ X, long ldx, int R, int Cn,
                                                             int KB, int shift, long sX, __bf16 *__restrict__ out,
                                                             long sOut) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, c0 = blockIdx.x * 64, kb = blockIdx.y;
  const float *x = X + (long)b * sX;
  const int t = threadIdx.x;
  if (((reinterpret_cast<unsigned long>(x) & 15) | (ldx & 3)) == 0) {  // 16 B per lane (as pack_cols_item)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int kr = (t >> 4) + 16 * i, cc = (t & 15) * 4;
      const int src = kb * 64 + kr - shift;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (kb * 64 + kr < R && src >= 0 && src < R) {
        const float *xr = x + (long)src * ldx + c0 + cc;
        if (c0 + cc + 3 < Cn) {
          v = *reinterpret_cast<const floatx4 *>(xr);
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++) v[e] = c0 + cc + e < Cn ? xr[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; e++) tile[kr][cc + e] = v[e];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int kr = (t >> 6) + 4 * i, cc = t & 63;
      const int src = kb * 64 + kr - shift;
      float v = 0.f;
      if (kb * 64 + kr < R && src >= 0 && src < R && c0 + cc < Cn) v = x[(long)src * ldx + c0 + cc];
      tile[kr][cc] = v;
    }
  }
  __syncthreads();
  const int c = t >> 2, part = t & 3;
  if (c0 + c >= Cn) return;
  __bf16 *o = out + (long)b * sOut + ((long)(c0 + c) * KB + kb) * 64 + part * 16;
  bf16x8 h0, h1;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    h0[j] = (__bf16)tile[part * 16 + j][c];
    h1[j] = (__bf16)tile[part * 16 + 8 + j][c];
  }
  *reinterpret_cast<bf16x8 *>(o) = h0;
  *reinterpret_cast<bf16x8 *>(o + 8) = h1;
}

}  // namespace

void bf16_pack_rows(hipStream_t s, const float *X, long ldx, int R, int K, __bf16 *out, int batch, long sX,
                    long sOut) {
  if (R <= 0 || K <= 0 || batch <= 0) return;
  const int KB = (K + 63) / 64;
  const int vec = ((uintptr_t)X % 16 == 0) && (ldx % 4 == 0) && (sX % 4 == 0);
  const dim3 grid(ceil_div(R, 4), batch);
  const int need = KB * 64;
  if (need <= 256) hipLaunchKernelGGL(bf16_pack_rows_kernel<1>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, vec);
  else if (need <= 512) hipLaunchKernelGGL(bf16_pack_rows_kernel<2>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, vec);
  else if (need <= 1024) hipLaunchKernelGGL(bf16_pack_rows_kernel<4>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, vec);
  else if (need <= 2048) hipLaunchKernelGGL(bf16_pack_rows_kernel<8>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, vec);
  else if (need <= 4096) hipLaunchKernelGGL(bf16_pack_rows_kernel<16>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, vec);
  else throw std::invalid_argument("bf16_pack_rows: K > 4096");
}

void bf16_pack_cols(hipStream_t s, const float *X, long ldx, int R, int Cn, int shift, __bf16 *out, int batch, long sX,
                    long sOut) {
  if (R <= 0 || Cn <= 0 || batch <= 0) return;
  const int KB = (R + 63) / 64;
  hipLaunchKernelGGL(bf16_pack_cols_kernel, dim3(ceil_div(Cn, 64), KB, batch), dim3(256), 0, s, X, ldx, R, Cn, KB,
                     shift, sX, out, sOut);
}

void x3p_pack_rows(hipStream_t s, const float *X, long ldx, int R, int K, _Float16 *out, int *eout, float bound,
                   int batch, long sX, long sOut, long sE) {
  if (R <= 0 || K <= 0 || batch <= 0) return;
  const int KB = (K + 31) / 32;
  const int vec = ((uintptr_t)X % 16 == 0) && (ldx % 4 == 0) && (sX % 4 == 0);
  const dim3 grid(ceil_div(R, 4), batch);
  // lanes cover KW*256 values of a row; the packed row also needs the zero pad up to KB*32
  const int need = KB * 32;
  if (need <= 256) hipLaunchKernelGGL(pack_rows_kernel<1>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, eout, sE, bound, vec);
  else if (need <= 512) hipLaunchKernelGGL(pack_rows_kernel<2>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, eout, sE, bound, vec);
  else if (need <= 1024) hipLaunchKernelGGL(pack_rows_kernel<4>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, eout, sE, bound, vec);
  else if (need <= 2048) hipLaunchKernelGGL(pack_rows_kernel<8>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, eout, sE, bound, vec);
  else if (need <= 4096) hipLaunchKernelGGL(pack_rows_kernel<16>, grid, dim3(256), 0, s, X, ldx, R, K, KB, sX, out, sOut, eout, sE, bound, vec);
  else throw std::invalid_argument("x3p_pack_rows: K > 4096");
}

void x3p_pack_cols(hipStream_t s, const float *X, long ldx, int R, int Cn, int shift, _Float16 *out, int *eout,
                   const unsigned *cmax, float bound, int batch, long sX, long sOut, long sE, long sCm,
                   const unsigned *avoid, int nxcd, int *counter) {
  if (R <= 0 || Cn <= 0 || batch <= 0) return;
  const int KB = (R + 31) / 32;
  if (avoid) {
    const long items = (long)ceil_div(Cn, 64) * ceil_div(KB, KPI) * batch;
    if (!counter || items + 8 >= (1L << 31)) throw std::invalid_argument("x3p_pack_cols: avoid needs a counter");
    hipLaunchKernelGGL(pack_cols_kernel, dim3((int)std::min<long>((items + 7) / 8, 1024)), dim3(256), 0, s, X, ldx, R,
                       Cn, KB, shift, sX, out, sOut, eout, sE, cmax, sCm, bound, avoid, nxcd, batch, counter);
    return;
  }
  hipLaunchKernelGGL(pack_cols_kernel, dim3(ceil_div(Cn, 64), ceil_div(KB, KPI), batch), dim3(256), 0, s, X, ldx, R,
                     Cn, KB, shift, sX, out, sOut, eout, sE, cmax, sCm, bound, nullptr, 0, batch, nullptr);
}

namespace {
// uniform [-1, 1) halves (fp16 or bf16 bit patterns) from a counter hash
__global__ void fill_halves_kernel(unsigned short *p, long n, unsigned seed, int bf16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    const float v = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    p[i] = bf16 ? __builtin_bit_cast(unsigned short, (__bf16)v) : __builtin_bit_cast(unsigned short, (_Float16)v);
  }
}
}  // namespace

float x3p_bench(hipStream_t s, int M, int N, int K, bool bf16, int iters, int split) {
  const int KB = bf16 ? (K + 63) / 64 : (K + 31) / 32;
  const long na = (long)M * KB * 64, nb = (long)N * KB * 64;
  _Float16 *A = nullptr, *B = nullptr;
  float *C = nullptr, *ws = nullptr;
  KCTC_HIP_CHECK(hipMalloc(&A, na * 2));
  KCTC_HIP_CHECK(hipMalloc(&B, nb * 2));
  KCTC_HIP_CHECK(hipMalloc(&C, (long)M * N * 4));
  if (split > 1) KCTC_HIP_CHECK(hipMalloc(&ws, (long)split * M * N * 4));
  hipLaunchKernelGGL(fill_halves_kernel, dim3(1024), dim3(256), 0, s, reinterpret_cast<unsigned short *>(A), na, 1u,
                     bf16 ? 1 : 0);
  hipLaunchKernelGGL(fill_halves_kernel, dim3(1024), dim3(256), 0, s, reinterpret_cast<unsigned short *>(B), nb, 2u,
                     bf16 ? 1 : 0);
  X3PArgs g;
  g.M = M; g.N = N; g.KB = KB; g.A = A; g.B = B; g.C = C; g.ldc = N; g.bf16 = bf16;
  g.split_k = split; g.ws = ws;
  for (int i = 0; i < 2; i++) gemm_x3p(s, g);
  hipEvent_t e0, e1;
  KCTC_HIP_CHECK(hipEventCreate(&e0));
  KCTC_HIP_CHECK(hipEventCreate(&e1));
  KCTC_HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; i++) gemm_x3p(s, g);
  KCTC_HIP_CHECK(hipEventRecord(e1, s));
  KCTC_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  KCTC_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
  (void)hipFree(A); (void)hipFree(B); (void)hipFree(C);
  if (ws) (void)hipFree(ws);
  return ms / iters;
}

static int env_backoff() { return 1; }

bool x3p_use_256(int M, int N) { return M >= 192 && N >= 192; }

int x3p_pick_split(int M, int N, int KB, int batch) {
  const int tb = x3p_use_256(M, N) ? TB2 : TB;
  const long tiles = (long)ceil_div(M, tb) * ceil_div(N, tb) * batch;
  if (tiles >= 384 || KB < 16) return 1;
  long want = (512 + tiles - 1) / tiles;
  want = std::min<long>(want, KB / 8);
  want = std::min<long>(want, 32);
  return want < 1 ? 1 : (int)want;
}

// kernel parameters of a gemm_x3p call (t256: it runs on 256 x 256 tiles)
static PParams x3p_params(const X3PArgs &g, bool &t256) {
  PParams p{};
  p.A = g.A; p.B = g.B; p.eA = g.eA; p.eB = g.eB; p.C = g.C; p.bias = g.bias; p.bias2 = g.bias2;
  p.ldc = g.ldc; p.sA = g.sA; p.sB = g.sB; p.sC = g.sC; p.sBias = g.sBias; p.seA = g.seA; p.seB = g.seB;
  p.M = g.M; p.N = g.N; p.KB = g.KB; p.alpha = g.alpha; p.beta = g.beta;
  p.gx = ceil_div(g.N, TB);
  p.tiles = p.gx * ceil_div(g.M, TB);
  p.batch = g.batch;
  p.split = (g.split_k > 1 && g.ws) ? g.split_k : 1;
  p.kbchunk = p.split > 1 ? ceil_div(g.KB, p.split) : (g.KB > 0 ? g.KB : 1);
  if (p.split > 1) p.split = ceil_div(g.KB, p.kbchunk);
  p.ws = g.ws;
  // large shapes on 256 x 256 tiles
  t256 = !g.stream_flags && x3p_use_256(g.M, g.N);
  if (t256) {
    p.gx = ceil_div(g.N, TB2);
    p.tiles = p.gx * ceil_div(g.M, TB2);
  }
  p.counter = g.tile_counter;
  p.eA0 = g.eA0; p.eB0 = g.eB0;
  p.sflags = g.stream_flags; p.snwg = g.stream_nwg; p.sT = g.stream_T; p.sN = g.stream_N;
  p.srg = g.stream_rg; p.sxg = g.stream_group_step;
  p.sgsh = g.stream_gs == 8 ? 3 : 4;
  p.backoff = env_backoff();
  p.nrt = ceil_div(g.M, TB);
  p.sxs = g.stream_step; p.serr = g.stream_err;
  p.xcd_word = g.stream_xcd_word; p.xcd_count = g.stream_xcd_count;
  p.sdir = 0;
  p.arrive = nullptr;
  p.mt = ceil_div(g.M, TB2);
  p.dbg = 0;
  p.p256v = 0;
  p.avoid = g.avoid_word;
  p.nxcd = g.avoid_xcds;
  if (p.avoid && (!t256 || !p.counter))
    throw std::invalid_argument("gemm_x3p: avoid_word needs a 256-tile launch with a tile counter");
  return p;
}

static void x3p_set_attrs() {
  static bool attr = false;  // dynamic LDS above 64 KB
  if (attr) return;
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_x3p_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBase));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_x3p_kernel<false, true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBase));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_x3p_kernel<true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsStream));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_x3p_kernel<true, true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsStream));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_p256_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds256));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_p256_kernel<true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds256));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_p256_pair_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds256));
  KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_p256_pair_kernel<true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds256));
  attr = true;
}

static void x3p_reduce(hipStream_t s, const PParams &p) {
  if (p.split <= 1) return;
  const long tot = (long)p.batch * p.M * p.N;
  hipLaunchKernelGGL(x3p_splitk_reduce, dim3((int)std::min<long>(2048, (tot + 255) / 256)), dim3(256), 0, s, p);
}

void gemm_x3p(hipStream_t s, const X3PArgs &g) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  if (g.stream_flags && !rnn_side_gated(s))
    throw std::logic_error("gemm_x3p: streaming launch beside a recurrence without its residency gate");
  bool t256 = false;
  PParams p = x3p_params(g, t256);
  const int total = p.tiles * p.batch * p.split;
  int blocks = total;
  if (g.max_blocks > 0 && total > g.max_blocks) blocks = std::max(8, g.max_blocks / 8 * 8);
  if (g.stream_flags && g.stream_arrive && g.stream_part && g.KB % 2 == 0 && (long)g.M * g.ldc * 4 + (long)(g.batch - 1) * g.sC * 4 < (1L << 31)) {
    p.sdir = 1;
    p.kbchunk = g.KB / 2;  // the producer's two directions
    p.arrive = g.stream_arrive;
    p.part = g.stream_part;
    KCTC_HIP_CHECK(hipMemsetAsync(p.arrive, 0, sizeof(int) * (size_t)stream_total(p) / 2, s));
  }
  if (p.counter) KCTC_HIP_CHECK(hipMemsetAsync(p.counter, 0, sizeof(int), s));
  x3p_set_attrs();
  if (t256) {
    if (g.bf16 && (p.eA || p.eB)) throw std::invalid_argument("gemm_x3p: bf16 operands take no exponents");
    if (g.bf16) hipLaunchKernelGGL(gemm_p256_kernel<true>, dim3(blocks), dim3(NTH2), kLds256, s, p);
    else hipLaunchKernelGGL(gemm_p256_kernel<false>, dim3(blocks), dim3(NTH2), kLds256, s, p);
  } else if (g.bf16 && !p.sflags) {
    if (p.eA || p.eB) throw std::invalid_argument("gemm_x3p: bf16 operands take no exponents");
    hipLaunchKernelGGL((gemm_x3p_kernel<false, true>), dim3(blocks), dim3(NTH), kLdsBase, s, p);
  } else if (p.sflags) {
    if (!p.counter || p.split > 1 || g.stream_N <= 0 || g.stream_step <= 0 ||
        (long)g.stream_T * g.stream_step * 2 >= (1L << 31))
      throw std::invalid_argument("gemm_x3p: bad streaming arguments");
    // persistent blocks, each owning its CU's LDS, so the producer's
    // workgroups always find free CUs (max_blocks = CUs left to this GEMM)
    const int sb = std::min(stream_total(p), g.max_blocks > 0 ? g.max_blocks : 176);
    if (g.bf16) {  // A: the producer's bf16 h images (same chunk addressing, 64 k per block)
      if (p.eB) throw std::invalid_argument("gemm_x3p: bf16 operands take no exponents");
      hipLaunchKernelGGL((gemm_x3p_kernel<true, true>), dim3(sb), dim3(NTH), kLdsStream, s, p);
    } else {
      hipLaunchKernelGGL(gemm_x3p_kernel<true>, dim3(sb), dim3(NTH), kLdsStream, s, p);
    }
    return;
  } else {
    hipLaunchKernelGGL(gemm_x3p_kernel<false>, dim3(blocks), dim3(NTH), kLdsBase, s, p);
  }
  x3p_reduce(s, p);
}

void gemm_x3p_pair(hipStream_t s, const X3PArgs &g1, const X3PArgs &g2) {
  if (g2.M <= 0 || g2.N <= 0 || g2.batch <= 0) return gemm_x3p(s, g1);
  if (g1.M <= 0 || g1.N <= 0 || g1.batch <= 0) return gemm_x3p(s, g2);
  bool a = false, b = false;
  PParams p = x3p_params(g1, a), q = x3p_params(g2, b);
  if (!a || !b || !p.counter || g1.bf16 != g2.bf16 || g1.stream_flags || g2.stream_flags)
    throw std::invalid_argument("gemm_x3p_pair: two 256-tile problems with a tile counter");
  if (g1.bf16 && (p.eA || p.eB || q.eA || q.eB)) throw std::invalid_argument("gemm_x3p: bf16 operands take no exponents");
  const int total = p.tiles * p.batch * p.split + q.tiles * q.batch * q.split;
  int blocks = total;
  if (g1.max_blocks > 0 && total > g1.max_blocks) blocks = std::max(8, g1.max_blocks / 8 * 8);
  KCTC_HIP_CHECK(hipMemsetAsync(p.counter, 0, sizeof(int), s));
  x3p_set_attrs();
  if (g1.bf16) hipLaunchKernelGGL(gemm_p256_pair_kernel<true>, dim3(blocks), dim3(NTH2), kLds256, s, p, q);
  else hipLaunchKernelGGL(gemm_p256_pair_kernel<false>, dim3(blocks), dim3(NTH2), kLds256, s, p, q);
  x3p_reduce(s, p);
  x3p_reduce(s, q);
}

size_t x3p_bwd_stream_ints(int M, int N) {
  const long nrt = ceil_div(M, TB), gx = ceil_div(N, TB);
  return (size_t)(1 + 2 * nrt + nrt * gx);
}

bool x3p_bwd_stream_256(int M, int N, int KB, bool bf16) {
  // per-tile buffer offsets stay below 2^31 (C rows are addressed as [M][ldc])
  return x3p_use_256(M, N) && KB * (bf16 ? 64 : 32) <= 4096;
}
// off by default: at configs[1] the streams end ~200 us after their
// producers with or without it (they run behind, not on the last jobs) and
// the extra partial traffic cost 1.4 % (752k vs 741k frames/s, same box)
int x3p_stream_tail_rows() { return 0; }
size_t x3p_bwd_stream_part2_floats(int N) {
  return (size_t)2 * x3p_stream_tail_rows() * ceil_div(N, TB2) * (kStreamTailSplit + 1) * TB2 * TB2;
}
size_t x3p_bwd_stream_part_floats(int M, int N) {
  return std::max((size_t)M * N, (size_t)ceil_div(M, TB2) * ceil_div(N, TB2) * TB2 * TB2);
}

void gemm_x3p_bwd_stream(hipStream_t s, const X3PBwdStream &a) {
  if (a.M <= 0 || a.N <= 0) return;
  if (!rnn_side_gated(s))
    throw std::logic_error("gemm_x3p_bwd_stream: streaming launch beside a recurrence without its residency gate");
  const int K = a.KB * (a.bf16 ? 64 : 32);
  if (K > 4096 || a.Nf <= 0 || (long)a.M * a.N * 4 >= (1L << 31) || (long)a.M * a.KB * 128 >= (1L << 31) ||
      (a.lde & 3) || (a.edoff & 3))
    throw std::invalid_argument("gemm_x3p_bwd_stream: unsupported shape");
  PParams p{};
  p.A = a.Ap; p.eA = a.eA; p.sA = (long)a.M * a.KB * 64; p.seA = a.M;
  p.B = a.B; p.eB = a.eB; p.sB = a.sB; p.seB = a.seB;
  p.C = a.C; p.ldc = a.ldc; p.alpha = 1.f; p.beta = 0.f;
  p.M = a.M; p.N = a.N; p.KB = a.KB;
  p.gx = ceil_div(a.N, TB); p.nrt = ceil_div(a.M, TB);
  p.tiles = p.gx * p.nrt; p.batch = 2; p.split = 1; p.kbchunk = a.KB;
  p.E = a.E; p.lde = a.lde; p.edoff = a.edoff;
  p.P = 4;
  p.counter = a.cnt; p.done = a.cnt + 1; p.arrive = a.cnt + 1 + 2 * p.nrt;
  p.part = a.part;
  p.sflags = a.flags; p.snwg = a.nwg; p.sT = a.T; p.sN = a.Nf; p.serr = a.err; p.srg = a.rg;
  p.xcd_word = a.xcd_word; p.xcd_count = a.xcd_count;
  p.backoff = env_backoff();
  p.dbg = 0;
  p.fwdp = a.forward ? 1 : 0;
  p.bias = a.bias; p.bias2 = a.bias2; p.bcols = a.bias_cols > 0 ? a.bias_cols : 1; p.sBias = a.sbias;
  const bool t256 = x3p_bwd_stream_256(a.M, a.N, a.KB, a.bf16);
  if ((a.forward || a.bias) && !t256) throw std::invalid_argument("gemm_x3p_bwd_stream: forward producer needs 256 tiles");
  KCTC_HIP_CHECK(hipMemsetAsync(a.cnt, 0, sizeof(int) * x3p_bwd_stream_ints(a.M, a.N), s));
  if (t256) {
    p.gx = ceil_div(a.N, TB2); p.nrt = ceil_div(a.M, TB2);
    p.tiles = p.gx * p.nrt;
    p.done = a.cnt + 1; p.arrive = a.cnt + 1 + 2 * p.nrt;  // within x3p_bwd_stream_ints (128-tile counts)
    const int tr = a.tail_rows >= 0 ? a.tail_rows : x3p_stream_tail_rows();
    p.tailr = a.part2 && tr > 0 && p.nrt >= 2 * tr + 2 ? tr : 0;
    p.tails = p.tailr ? kStreamTailSplit : 1;
    p.part2 = a.part2;
    const int total = 2 * (p.nrt - p.tailr) * (p.P + p.gx) + 2 * p.tailr * (p.P + p.gx * p.tails);
    const dim3 grid(std::min(total, a.blocks > 0 ? a.blocks : 96));
    auto go = [&](auto kern) {
      static bool attr = false;
      if (!attr) {
        KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds256));
        attr = true;
      }
      hipLaunchKernelGGL(kern, grid, dim3(NTH2), kLds256, s, p);
    };
    if (a.bf16) {
      if (K <= 1024) go(x3p_bwd_stream256_kernel<4, true>);
      else if (K <= 2048) go(x3p_bwd_stream256_kernel<8, true>);
      else go(x3p_bwd_stream256_kernel<16, true>);
    } else {
      if (K <= 1024) go(x3p_bwd_stream256_kernel<4, false>);
      else if (K <= 2048) go(x3p_bwd_stream256_kernel<8, false>);
      else go(x3p_bwd_stream256_kernel<16, false>);
    }
    return;
  }
  const int total = 2 * p.nrt * (p.P + p.gx);
  const dim3 grid(std::min(total, a.blocks > 0 ? a.blocks : 96));
  auto go = [&](auto kern) {
    static bool attr = false;
    if (!attr) {
      KCTC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsStream));
      attr = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(NTH), kLdsStream, s, p);
  };
  if (a.bf16) {
    if (K <= 1024) go(x3p_bwd_stream_kernel<4, true>);
    else if (K <= 2048) go(x3p_bwd_stream_kernel<8, true>);
    else go(x3p_bwd_stream_kernel<16, true>);
  } else {
    if (K <= 1024) go(x3p_bwd_stream_kernel<4, false>);
    else if (K <= 2048) go(x3p_bwd_stream_kernel<8, false>);
    else go(x3p_bwd_stream_kernel<16, false>);
  }
}

void x3p_row_stream_selftest(hipStream_t s, int M, int N, int KB, int forward, int tail_rows, const float *E,
                             const float *Wt, const float *bias, float *C) {
  const int K = KB * 32, Nf = 16, T = (M + Nf - 1) / Nf;
  if (M <= 0 || N <= 0 || KB <= 0 || M % Nf) throw std::invalid_argument("x3p_row_stream_selftest: shape");
  if (!x3p_bwd_stream_256(M, N, KB, false)) throw std::invalid_argument("x3p_row_stream_selftest: not a 256-tile shape");
  const int tr = tail_rows >= 0 ? tail_rows : x3p_stream_tail_rows();
  const size_t ap = (size_t)2 * M * KB * 128, bp = (size_t)2 * N * KB * 128;
  const size_t part = sizeof(float) * x3p_bwd_stream_part_floats(M, N);
  const size_t part2 = sizeof(float) * (size_t)2 * tr * ceil_div(N, TB2) * (kStreamTailSplit + 1) * TB2 * TB2;
  const size_t cnt = sizeof(int) * x3p_bwd_stream_ints(M, N), fl = 4096;
  char *buf = nullptr;
  const size_t total = ap + bp + part + part2 + cnt + fl + sizeof(int) * 4 * (size_t)(M + N) + 4096;
  KCTC_HIP_CHECK(hipMalloc(&buf, total));
  char *o = buf;
  auto take = [&](size_t b) { char *r = o; o += (b + 255) / 256 * 256; return r; };
  _Float16 *A = reinterpret_cast<_Float16 *>(take(ap)), *B = reinterpret_cast<_Float16 *>(take(bp));
  float *pt = reinterpret_cast<float *>(take(part)), *pt2 = reinterpret_cast<float *>(take(part2));
  int *cn = reinterpret_cast<int *>(take(cnt));
  unsigned *flags = reinterpret_cast<unsigned *>(take(fl));
  int *eA = reinterpret_cast<int *>(take(sizeof(int) * 2 * (size_t)M)), *eB = reinterpret_cast<int *>(take(sizeof(int) * 2 * (size_t)N));
  // every epoch final: lines (d) at 32-word strides
  std::vector<unsigned> hf(fl / 4, (unsigned)(T + 2));
  hf[1000] = 0u;  // the error word
  KCTC_HIP_CHECK(hipMemcpyAsync(flags, hf.data(), fl, hipMemcpyHostToDevice, s));
  x3p_pack_rows(s, Wt, K, N, K, B, eB, 0.f, 2, (long)N * K, (long)N * KB * 64, N);
  X3PBwdStream a;
  a.M = M; a.N = N; a.KB = KB;
  a.E = E; a.lde = 2L * K; a.edoff = K;
  a.Ap = A; a.eA = eA;
  a.B = B; a.eB = eB; a.sB = (long)N * KB * 64; a.seB = N;
  a.C = C; a.ldc = N;
  a.part = pt; a.part2 = tr > 0 ? pt2 : nullptr; a.tail_rows = tr; a.cnt = cn;
  a.flags = flags; a.nwg = 1; a.T = T; a.Nf = Nf; a.err = flags + 1000; a.rg = 1;
  a.blocks = 64;
  a.forward = forward != 0;
  a.bias = bias; a.bias_cols = N;
  gemm_x3p_bwd_stream(s, a);
  KCTC_HIP_CHECK(hipStreamSynchronize(s));
  unsigned err = 0;
  KCTC_HIP_CHECK(hipMemcpy(&err, flags + 1000, sizeof(unsigned), hipMemcpyDeviceToHost));
  KCTC_HIP_CHECK(hipFree(buf));
  if (err) throw std::runtime_error("x3p_row_stream_selftest: wait timeout");
}

}  // namespace kctc
