// gemm.hip -- fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_16x16x4_f32).
//
// Tile 128x128x32, 256 threads = 4 waves in a 2x2 grid, each wave owns a 64x64
// sub-tile = 4x4 MFMA tiles (64 accumulator VGPRs).  Both operands are staged
// through LDS in a "k-contiguous" image ([row][k], padded to 36 floats so the
// 16 rows a ds_read_b128 lane group touches fall on distinct 16-B slots),
// register-staged and double-buffered: the next K-tile's global loads are in
// flight while the current tile is multiplied, one barrier per K-tile.
//
// The K index inside each 16-wide group is permuted (lane quad q handles
// k = 4q..4q+3 over the 4 MFMA k-steps) so that every lane fetches its four
// k-step operands with ONE ds_read_b128; the sum is over all k either way and
// v_mfma_f32_16x16x4_f32 is an exact fp32 FMA chain.
//
// Block -> tile mapping is XCD-aware (blocks that share an XCD get adjacent
// tiles along N, so they share A row panels in that XCD's L2).  Split-K writes
// fp32 slabs that a second kernel reduces in a fixed order (deterministic).
#include "common.h"
#include "gemm.h"

namespace kctc {
namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDK = BK + 4, NT = 256;
// LDS image per operand: "k-contiguous" [row][LDK] when the source is
// k-contiguous (A row-major, B^T row-major), else "row-contiguous" [BK][LDM]
// so that the 16-B global loads land with one ds_write_b128 instead of four
// scalar transposing writes; fragments are then read with 4 ds_read_b32
// (conflict-free: LDM = 132 puts lane groups fq=0/1 on bank halves 0-15/16-31).
constexpr int LDM = BM + 4;
constexpr int OPSZ = (BM * LDK > BK * LDM) ? BM * LDK : BK * LDM;
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct KParams {
  const float *A, *B;
  float *C;
  const float *bias, *bias2;
  long lda, ldb, ldc;
  long strideA, strideB, strideC, strideBias;
  int M, N, K, gx, tiles, batch, split, kchunk;
  float alpha, beta;
  float *ws;
  int vecA, vecB;
  int *counter;
};

// Load one operand tile (rows r0.., k0..) into 4 float4 registers.
//   KC (k-contiguous source): elem(r,k) = P[r*ld + k]
//   else (r-contiguous source): elem(r,k) = P[k*ld + r]
template <bool KC>
__device__ __forceinline__ void load_tile(const float *__restrict__ P, long ld, int rows, int r0,
                                          int k0, int kend, int vec, floatx4 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    int r, k;
    if (KC) { r = r0 + (t >> 3) + 32 * i; k = k0 + (t & 7) * 4; }
    else    { k = k0 + (t >> 5) + 8 * i;  r = r0 + (t & 31) * 4; }
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (KC) {
      if (r < rows) {
        const float *p = P + (long)r * ld + k;
        if (vec && k + 3 < kend) {
          v = *reinterpret_cast<const floatx4 *>(p);
        } else {
#pragma unroll
          for (int j = 0; j < 4; j++) v[j] = (k + j < kend) ? p[j] : 0.f;
        }
      }
    } else {
      if (k < kend) {
        const float *p = P + (long)k * ld + r;
        if (vec && r + 3 < rows) {
          v = *reinterpret_cast<const floatx4 *>(p);
        } else {
#pragma unroll
          for (int j = 0; j < 4; j++) v[j] = (r + j < rows) ? p[j] : 0.f;
        }
      }
    }
    reg[i] = v;
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(float *__restrict__ S, const floatx4 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (KC) {
      int r = (t >> 3) + 32 * i, k = (t & 7) * 4;
      *reinterpret_cast<floatx4 *>(S + r * LDK + k) = reg[i];
    } else {
      int k = (t >> 5) + 8 * i, r = (t & 31) * 4;
      *reinterpret_cast<floatx4 *>(S + k * LDM + r) = reg[i];
    }
  }
}

template <bool KC>
__device__ __forceinline__ floatx4 frag(const float *S, int row, int k0) {
  if (KC) return *reinterpret_cast<const floatx4 *>(S + row * LDK + k0);
  return floatx4{S[(k0 + 0) * LDM + row], S[(k0 + 1) * LDM + row], S[(k0 + 2) * LDM + row],
                 S[(k0 + 3) * LDM + row]};
}

template <bool TA, bool TB>
__device__ __forceinline__ void gemm_tile(const KParams &p, float (&lds)[2][2 * OPSZ], int id, int total,
                                          bool remap) {
  // XCD-aware bijective remap of the work index (id & 7 is the XCD as long as
  // the grid is a multiple of 8 or covers all work items); dynamic ids are
  // handed out in time order and used as they are
  const int q = total >> 3, rr = total & 7, xcd = id & 7, loc = id >> 3;
  const int wl = remap ? (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc : id;
  const int bz = wl / p.tiles, wg = wl - bz * p.tiles;
  const int tn = wg % p.gx, tm = wg / p.gx;
  const int b = bz % p.batch, ks = bz / p.batch;
  const float *A = p.A + (long)b * p.strideA;
  const float *B = p.B + (long)b * p.strideB;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int fr = lane & 15, fq = lane >> 4;

  // A operand: rows m; KC iff !TA.  B operand: rows n; KC iff TB.
  const float *Ab = TA ? A + m0 : A + (long)m0 * p.lda;
  const float *Bb = TB ? B + (long)n0 * p.ldb : B + n0;
  const int arows = p.M - m0, brows = p.N - n0;

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  floatx4 ra[4], rb[4];
  int nk = (kend - kbeg + BK - 1) / BK;
  if (nk < 0) nk = 0;
  if (nk > 0) {
    load_tile<!TA>(Ab, p.lda, arows, 0, kbeg, kend, p.vecA, ra);
    load_tile<TB>(Bb, p.ldb, brows, 0, kbeg, kend, p.vecB, rb);
    store_tile<!TA>(lds[0], ra);
    store_tile<TB>(lds[0] + OPSZ, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<!TA>(Ab, p.lda, arows, 0, k0, kend, p.vecA, ra);
      load_tile<TB>(Bb, p.ldb, brows, 0, k0, kend, p.vecB, rb);
    }
    const float *sA = lds[cur], *sB = lds[cur] + OPSZ;
#pragma unroll
    for (int kg = 0; kg < BK / 16; kg++) {
      floatx4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; i++) fa[i] = frag<!TA>(sA, wm + i * 16 + fr, kg * 16 + fq * 4);
#pragma unroll
      for (int j = 0; j < 4; j++) fb[j] = frag<TB>(sB, wn + j * 16 + fr, kg * 16 + fq * 4);
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int j = 0; j < 4; j++)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<!TA>(lds[cur ^ 1], ra);
      store_tile<TB>(lds[cur ^ 1] + OPSZ, rb);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> C[m0+wm+16i+4fq+r][n0+wn+16j+fr]
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
          if (row < p.M) W[(long)row * p.N + col] = acc[i][j][r];
        }
      }
    return;
  }
  float *C = p.C + (long)b * p.strideC;
  const float *bias = p.bias ? p.bias + (long)b * p.strideBias : nullptr;
  const float *bias2 = p.bias2 ? p.bias2 + (long)b * p.strideBias : nullptr;
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
          float v = p.alpha * acc[i][j][r] + badd;
          if (p.beta != 0.f) v += p.beta * *c;
          *c = v;
        }
      }
    }
}

// One work item = (tile, batch, k-slab).  The grid either covers every item or
// (max_blocks) is a persistent multiple of 8 that strides over them, leaving
// CUs free for a concurrently running recurrence.
template <bool TA, bool TB>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(KParams p) {
  __shared__ __attribute__((aligned(16))) float lds[2][2 * OPSZ];
  __shared__ int next;
  const int total = p.tiles * p.batch * p.split;
  if (p.counter) {
    while (true) {
      if (threadIdx.x == 0) next = atomicAdd(p.counter, 1);
      __syncthreads();
      const int id = next;
      __syncthreads();
      if (id >= total) break;
      gemm_tile<TA, TB>(p, lds, id, total, false);
    }
    return;
  }
  for (int id = blockIdx.x; id < total; id += gridDim.x) gemm_tile<TA, TB>(p, lds, id, total, true);
}

// max |x| per row (rows < nrows, cols < ncols) into rmax[b][row] (float bits),
// and per column, atomically max-merged into cmax[b][col] (pre-zeroed); either
// output may be null.  One wave per (row, 64-column group) pass.
__global__ __launch_bounds__(256) void absmax_kernel(const float *__restrict__ X, long ldx, int nrows, int ncols,
                                                     long strideX, unsigned *__restrict__ rmax,
                                                     unsigned *__restrict__ cmax, long strideR, long strideC,
                                                     int rows_per_block) {
  const int b = blockIdx.y;
  const float *x = X + (long)b * strideX;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(nrows, r0 + rows_per_block);
  __shared__ float cm[4][1024];
  for (int c0 = 0; c0 < ncols; c0 += 1024) {
    float colm[16];
#pragma unroll
    for (int j = 0; j < 16; j++) colm[j] = 0.f;
    for (int r = r0 + w; r < r1; r += 4) {
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int c = c0 + j * 64 + lane;
        const float v = c < ncols ? fabsf(x[(long)r * ldx + c]) : 0.f;
        m = fmaxf(m, v);
        colm[j] = fmaxf(colm[j], v);
      }
      if (rmax) {
        m = wave_max(m);
        if (lane == 0) {
          if (c0 == 0) rmax[(long)b * strideR + r] = __float_as_uint(m);
          else atomicMax(rmax + (long)b * strideR + r, __float_as_uint(m));
        }
      }
    }
    if (cmax) {
#pragma unroll
      for (int j = 0; j < 16; j++) cm[w][j * 64 + lane] = colm[j];
      __syncthreads();
      for (int c = threadIdx.x; c < 1024 && c0 + c < ncols; c += 256) {
        const float m = fmaxf(fmaxf(cm[0][c], cm[1][c]), fmaxf(cm[2][c], cm[3][c]));
        atomicMax(cmax + (long)b * strideC + c0 + c, __float_as_uint(m));
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce(KParams p) {
  const long total = (long)p.batch * p.M * p.N;
  const long MN = (long)p.M * p.N;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int b = (int)(e / MN);
    const long rem = e - (long)b * MN;
    const int row = (int)(rem / p.N), col = (int)(rem - (long)row * p.N);
    float s = 0.f;
    for (int k = 0; k < p.split; k++) s += p.ws[((long)k * p.batch + b) * MN + rem];
    float *c = p.C + (long)b * p.strideC + (long)row * p.ldc + col;
    float v = p.alpha * s;
    if (p.bias) v += p.bias[(long)b * p.strideBias + col];
    if (p.bias2) v += p.bias2[(long)b * p.strideBias + col];
    if (p.beta != 0.f) v += p.beta * *c;
    *c = v;
  }
}

__global__ __launch_bounds__(256) void colsum_kernel(const float *__restrict__ X, long ldx, int rows,
                                                     int cols, float alpha, float beta,
                                                     float *__restrict__ out, long strideX,
                                                     long strideOut) {
  __shared__ float part[4][64];
  const int b = blockIdx.y, c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const float *x = X + (long)b * strideX;
  float s = 0.f;
  if (c < cols)
    for (int r = g; r < rows; r += 4) s += x[(long)r * ldx + c];
  part[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < cols) {
    float v = ((part[0][threadIdx.x] + part[1][threadIdx.x]) + part[2][threadIdx.x]) + part[3][threadIdx.x];
    float *o = out + (long)b * strideOut + c;
    *o = alpha * v + (beta != 0.f ? beta * *o : 0.f);
  }
}

}  // namespace

int gemm_pick_split(int M, int N, int K, int batch) {
  const long tiles = (long)ceil_div(M, BM) * ceil_div(N, BN) * batch;
  if (tiles >= 192 || K < 4 * BK) return 1;
  long want = (256 + tiles - 1) / tiles;
  long maxs = K / (2 * BK);
  if (want > maxs) want = maxs;
  if (want > 64) want = 64;
  return want < 1 ? 1 : (int)want;
}

void gemm_f32(hipStream_t stream, const GemmArgs &g) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  KParams p;
  p.A = g.A; p.B = g.B; p.C = g.C; p.bias = g.bias; p.bias2 = g.bias2;
  p.lda = g.lda; p.ldb = g.ldb; p.ldc = g.ldc;
  p.strideA = g.strideA; p.strideB = g.strideB; p.strideC = g.strideC; p.strideBias = g.strideBias;
  p.M = g.M; p.N = g.N; p.K = g.K; p.alpha = g.alpha; p.beta = g.beta;
  p.gx = ceil_div(g.N, BN);
  p.tiles = p.gx * ceil_div(g.M, BM);
  p.batch = g.batch;
  p.split = (g.split_k > 1 && g.ws) ? g.split_k : 1;
  p.kchunk = p.split > 1 ? (int)align_up((size_t)ceil_div(g.K, p.split), BK) : (g.K > 0 ? g.K : 1);
  if (p.split > 1) p.split = ceil_div(g.K, p.kchunk);
  p.ws = g.ws;
  auto aligned = [](const void *ptr, long ld, long stride) {
    return ((uintptr_t)ptr % 16 == 0) && (ld % 4 == 0) && (stride % 4 == 0);
  };
  p.vecA = aligned(g.A, g.lda, g.strideA);
  p.vecB = aligned(g.B, g.ldb, g.strideB);
  const int total = p.tiles * p.batch * p.split;
  int blocks = total;
  if (g.max_blocks > 0 && total > g.max_blocks) blocks = std::max(8, g.max_blocks / 8 * 8);
  p.counter = g.tile_counter;
  if (p.counter) KCTC_HIP_CHECK(hipMemsetAsync(p.counter, 0, sizeof(int), stream));
  dim3 grid(blocks);
  if (!g.transA && !g.transB) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, dim3(NT), 0, stream, p);
  else if (!g.transA && g.transB) hipLaunchKernelGGL((gemm_kernel<false, true>), grid, dim3(NT), 0, stream, p);
  else if (g.transA && !g.transB) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, dim3(NT), 0, stream, p);
  else hipLaunchKernelGGL((gemm_kernel<true, true>), grid, dim3(NT), 0, stream, p);
  if (p.split > 1) {
    long total = (long)p.batch * p.M * p.N;
    int blocks = (int)std::min<long>(2048, (total + 255) / 256);
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, stream, p);
  }
}

void absmax_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, unsigned *rmax, unsigned *cmax,
                int batch, long strideX, long strideR, long strideC) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return;
  if (cmax) KCTC_HIP_CHECK(hipMemsetAsync(cmax, 0, sizeof(unsigned) * (size_t)(batch > 1 ? strideC * (batch - 1) + cols : cols), stream));
  const int rpb = 64;
  hipLaunchKernelGGL(absmax_kernel, dim3(ceil_div(rows, rpb), batch), dim3(256), 0, stream, X, ldx, rows, cols,
                     strideX, rmax, cmax, strideR, strideC, rpb);
}

void colsum_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, float alpha,
                float beta, float *out, int batch, long strideX, long strideOut) {
  if (cols <= 0 || batch <= 0) return;
  hipLaunchKernelGGL(colsum_kernel, dim3(ceil_div(cols, 64), batch), dim3(256), 0, stream, X, ldx,
                     rows, cols, alpha, beta, out, strideX, strideOut);
}

}  // namespace kctc
