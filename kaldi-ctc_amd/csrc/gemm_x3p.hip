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

#include "common.h"
#include "gemm.h"

namespace kctc {
namespace {

constexpr int TB = 128;          // tile rows (M) = tile cols (N)
constexpr int NTH = 256;
constexpr int ROWB = 128;        // bytes per packed row block (64 halves)
constexpr int TILEB = TB * ROWB; // 16 KB per operand tile per stage
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));

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
};

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
    __builtin_amdgcn_global_load_lds(src, dst + q * 1024, 16, 0, 0);
  }
}

__device__ __forceinline__ halfx8 frag(const unsigned char *tile, int row, int chunk) {
  return *reinterpret_cast<const halfx8 *>(tile + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

__device__ void x3p_tile(const PParams &p, unsigned char *lds, int id, int total, bool remap) {
  const int q = total >> 3, rr = total & 7, xcd = id & 7, loc = id >> 3;
  const int wl = remap ? (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc : id;
  const int bz = wl / p.tiles, wg = wl - bz * p.tiles;
  const int tn = wg % p.gx, tm = wg / p.gx;
  const int b = bz % p.batch, ks = bz / p.batch;
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

  // LDS: [2 stages][A tile | B tile]
  if (nk > 0) {
    issue_tile(A, p.M, m0, p.KB, kb0, lds);
    issue_tile(B, p.N, n0, p.KB, kb0, lds + TILEB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; it++) {
    unsigned char *cur = lds + (it & 1) * 2 * TILEB;
    if (it + 1 < nk) {
      unsigned char *nxt = lds + ((it + 1) & 1) * 2 * TILEB;
      issue_tile(A, p.M, m0, p.KB, kb0 + it + 1, nxt);
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> C[m0+wm+16i+4fq+r][n0+wn+16j+fr], times 2^-(eA + eB)
  const int *eA = p.eA + (long)b * p.seA;
  const int *eB = p.eB + (long)b * p.seB;
  int eb[4], ea[4][4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int col = n0 + wn + j * 16 + fr;
    eb[j] = col < p.N ? eB[col] : 0;
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = m0 + wm + i * 16 + fq * 4 + r;
      ea[i][r] = row < p.M ? eA[row] : 0;
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

__global__ __launch_bounds__(NTH, 2) void gemm_x3p_kernel(PParams p) {
  // ONE shared array (a second __shared__ object can make hipcc wait vmcnt(0)
  // before LDS reads while a DMA is in flight)
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILEB + 16];
  int *next = reinterpret_cast<int *>(lds + 2 * 2 * TILEB);
  const int total = p.tiles * p.batch * p.split;
  if (p.counter) {
    while (true) {
      if (threadIdx.x == 0) *next = atomicAdd(p.counter, 1);
      __syncthreads();
      const int id = *next;
      __syncthreads();
      if (id >= total) break;
      x3p_tile(p, lds, id, total, false);
    }
    return;
  }
  for (int id = blockIdx.x; id < total; id += gridDim.x) x3p_tile(p, lds, id, total, true);
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

// Column packing (transpose): packed row c = column c of X, K = X's rows
// (k -> X row k - shift, zero outside [0, R)).  Exponent from cmax[c] (max |x|
// of the column, float bits) or the bound.  Block: 64 columns x one 32-k block.
__global__ __launch_bounds__(256) void pack_cols_kernel(const float *__restrict__ X, long ldx, int R, int Cn, int KB,
                                                        int shift, long sX, _Float16 *__restrict__ out, long sOut,
                                                        int *__restrict__ eout, long sE,
                                                        const unsigned *__restrict__ cmax, long sCm, float bound) {
  __shared__ float tile[32][65];
  const int b = blockIdx.z, c0 = blockIdx.x * 64, kb = blockIdx.y;
  const float *x = X + (long)b * sX;
  const int t = threadIdx.x;
  // load 32 rows x 64 columns (each row: 64 consecutive floats)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int kr = (t >> 6) + 4 * i, cc = t & 63;
    const int src = kb * 32 + kr - shift;
    float v = 0.f;
    if (kb * 32 + kr < R && src >= 0 && src < R && c0 + cc < Cn) v = x[(long)src * ldx + c0 + cc];
    tile[kr][cc] = v;
  }
  __syncthreads();
  const int c = t >> 2, part = t & 3;
  if (c0 + c >= Cn) return;
  const int e = bound > 0.f ? split_exp_d(bound)
                            : split_exp_d(__uint_as_float(cmax[(long)b * sCm + c0 + c]));
  halfx8 h, l;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const float xv = ldexpf(tile[part * 8 + j][c], e);
    h[j] = (_Float16)xv;
    l[j] = (_Float16)(xv - (float)h[j]);
  }
  _Float16 *o = out + (long)b * sOut + ((long)(c0 + c) * KB + kb) * 64;
  *reinterpret_cast<halfx8 *>(o + part * 8) = h;
  *reinterpret_cast<halfx8 *>(o + 32 + part * 8) = l;
  if (kb == 0 && part == 0 && eout) eout[(long)b * sE + c0 + c] = e;
}

}  // namespace

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
                   const unsigned *cmax, float bound, int batch, long sX, long sOut, long sE, long sCm) {
  if (R <= 0 || Cn <= 0 || batch <= 0) return;
  const int KB = (R + 31) / 32;
  hipLaunchKernelGGL(pack_cols_kernel, dim3(ceil_div(Cn, 64), KB, batch), dim3(256), 0, s, X, ldx, R, Cn, KB, shift,
                     sX, out, sOut, eout, sE, cmax, sCm, bound);
}

void gemm_x3p(hipStream_t s, const X3PArgs &g) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  PParams p;
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
  const int total = p.tiles * p.batch * p.split;
  int blocks = total;
  if (g.max_blocks > 0 && total > g.max_blocks) blocks = std::max(8, g.max_blocks / 8 * 8);
  p.counter = g.tile_counter;
  if (p.counter) KCTC_HIP_CHECK(hipMemsetAsync(p.counter, 0, sizeof(int), s));
  hipLaunchKernelGGL(gemm_x3p_kernel, dim3(blocks), dim3(NTH), 0, s, p);
  if (p.split > 1) {
    const long tot = (long)p.batch * p.M * p.N;
    hipLaunchKernelGGL(x3p_splitk_reduce, dim3((int)std::min<long>(2048, (tot + 255) / 256)), dim3(256), 0, s, p);
  }
}

}  // namespace kctc
