// gemm.h -- fp32 MFMA GEMM for gfx950 (v_mfma_f32_16x16x4_f32, exact fp32).
// Replaces the cublasSgemm calls of the reference's CuMatrix::AddMatMat
// (src/cudamatrix/cu-matrix.cc:1077-1110) and cuDNN's internal gate GEMMs.
#pragma once
#include <hip/hip_runtime.h>

namespace kctc {

// Row-major: C[b][i][j] = alpha * sum_k opA(b,i,k) opB(b,k,j) + beta * C[b][i][j]
//                         (+ bias[b][j] + bias2[b][j] when given)
//   opA(i,k) = transA ? A[k*lda + i] : A[i*lda + k]
//   opB(k,j) = transB ? B[j*ldb + k] : B[k*ldb + j]
// Batch strides may be negative.  split_k > 1 needs `ws` of
// split_k * batch * M * N floats and makes the result deterministic (slab
// reduce in fixed order).
struct GemmArgs {
  bool transA = false, transB = false;
  int M = 0, N = 0, K = 0;
  float alpha = 1.f, beta = 0.f;
  const float *A = nullptr, *B = nullptr;
  float *C = nullptr;
  long lda = 0, ldb = 0, ldc = 0;
  const float *bias = nullptr, *bias2 = nullptr;
  int batch = 1;
  long strideA = 0, strideB = 0, strideC = 0, strideBias = 0;
  int split_k = 1;
  float *ws = nullptr;
  int max_blocks = 0;  // > 0: persistent grid of at most this many workgroups
  // optional: zeroed device int -> dynamic tile scheduling (blocks pull work
  // items from this counter; blocks that start late, e.g. on CUs a concurrent
  // persistent kernel holds, find the work done and exit)
  int *tile_counter = nullptr;
};

void gemm_f32(hipStream_t stream, const GemmArgs &g);
// Heuristic split-K so that tiles * split fill the chip; returns 1 if not needed.
int gemm_pick_split(int M, int N, int K, int batch);

// max |X| per row (rmax[b][r]) and per column (cmax[b][c]) as float bits; either may be null
void absmax_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, unsigned *rmax, unsigned *cmax,
                int batch = 1, long strideX = 0, long strideR = 0, long strideC = 0);

// Split-fp16 GEMM on packed operands (gemm_x3p.hip).  Packed operand:
// [rows][KB][64] fp16 = per 32-k block 32 hi then 32 lo halves of the row
// scaled by 2^e[row]; e[] int per row.  C[b][m][n] = alpha 2^-(eA[m]+eB[n])
// sum_k A[m][k] B[n][k] (+ beta C + bias[n] + bias2[n]).
struct X3PArgs {
  int M = 0, N = 0, KB = 0;
  const _Float16 *A = nullptr, *B = nullptr;
  const int *eA = nullptr, *eB = nullptr;
  float *C = nullptr;
  long ldc = 0;
  float alpha = 1.f, beta = 0.f;
  const float *bias = nullptr, *bias2 = nullptr;
  int batch = 1;
  long sA = 0, sB = 0, sC = 0, sBias = 0, seA = 0, seB = 0;
  int split_k = 1;
  float *ws = nullptr;  // split_k * batch * M * N floats
  int max_blocks = 0;
  int *tile_counter = nullptr;
  int eA0 = 0, eB0 = 0;  // exponents used when eA / eB is null
  // Streaming mode (stream_flags != null): the A rows are frames (t, n),
  // row = t * stream_N + n, produced by a concurrently running bidirectional
  // v6 forward recurrence; a row tile is computed only once direction 0 has
  // published step t_max of the tile and direction 1 step T-1-t_min (flag
  // lines of rnn.hip: word 32 * (d * nwg + g) holds the WG's epoch = step + 2).
  // A is the producer's exchange-image array, read in place with sc1 loads
  // (eA0 = 14, KB over both directions).  Row tiles are taken in readiness order.
  // tile_counter is required; the grid must leave >= 64 CUs to the producer.
  const unsigned *stream_flags = nullptr;
  int stream_nwg = 0, stream_T = 0, stream_N = 0;
  long stream_step = 0;              // halves per producer step image (A = image of step 0)
  int stream_rg = 1;                  // producer row groups (N > 16): flags and image parts per group
  int stream_gs = 16;                 // sequences per producer row group (16 or 8)
  // direction-split streaming (gemm_x3p_kernel's fwd_combine): [row tiles][batch][col tiles]
  // zeroed ints; null: whole-K jobs after both directions' rows are in
  int *stream_arrive = nullptr;
  float *stream_part = nullptr;         // [row tiles][batch][col tiles][128 x 128] half-K partials
  long stream_group_step = 0;         // halves per row group's part of a step image
  unsigned *stream_err = nullptr;    // set (bit 2) if the producer stops publishing
  // XCD-pinned producer (rnn.hip xcd_mask): blocks on its XCDs exit before
  // taking work, as in X3PBwdStream
  const unsigned *stream_xcd_word = nullptr;
  int stream_xcd_count = 0;
  // bf16 operands (bf16_pack_rows / _cols: [rows][KB][64] bf16, KB = 64-k
  // blocks, no exponents): two v_mfma_f32_16x16x32_bf16 per stage, fp32
  // accumulation; streaming: A = a bf16 v6 forward's h images (eA0 = 0)
  bool bf16 = false;
  // Beside an XCD-pinned recurrence (non-gated, non-streaming 256-tile GEMMs
  // with a tile counter): blocks whose XCD has its bit set in *avoid_word
  // (rnn.hip rnn_pinned_xcds: the XCDs pinned backward recurrences ran on)
  // exit before taking work, so no block ever holds a CU the recurrence
  // needs and the launch ends when the other XCDs' blocks run out of tiles
  // (no block exits while the word names all avoid_xcds XCDs of the device:
  // then no XCD is left to the GEMM's tiles)
  const unsigned *avoid_word = nullptr;
  int avoid_xcds = 8;
};
void gemm_x3p(hipStream_t s, const X3PArgs &g);
// rnn.hip: s passed the residency gate of the recurrence in flight (or none is)
bool rnn_side_gated(hipStream_t s);
// two independent 256-tile problems (e.g. a layer's dW and dR) as ONE launch
// sharing g1's tile counter, then each one's split-K reduction: beside a
// pinned recurrence a launch completes only once its blocks on the
// recurrence's XCDs could start, so one launch per recurrence keeps the
// side stream from falling a GEMM behind per layer
void gemm_x3p_pair(hipStream_t s, const X3PArgs &g1, const X3PArgs &g2);
// shapes gemm_x3p runs on 256 x 256 tiles
bool x3p_use_256(int M, int N);
// split-K for gemm_x3p on a (M x N, KB k-blocks, batch) problem so that the
// tiles fill the chip (callers size ws for it: split * batch * M * N floats)
int x3p_pick_split(int M, int N, int KB, int batch);
// ms per gemm_x3p on random packed operands (M x K times N x K), iters launches
float x3p_bench(hipStream_t s, int M, int N, int K, bool bf16, int iters, int split);
// bf16-packed operands for gemm_x3p(bf16): rows (out[b][r][KB][64], KB =
// ceil(K / 64)) and columns (the transpose, source row k - shift), zero pad
void bf16_pack_rows(hipStream_t s, const float *X, long ldx, int R, int K, __bf16 *out, int batch = 1, long sX = 0,
                    long sOut = 0);
void bf16_pack_cols(hipStream_t s, const float *X, long ldx, int R, int Cn, int shift, __bf16 *out, int batch = 1,
                    long sX = 0, long sOut = 0);

// C = sum over the two directions d of A_d B_d^T, where A_d = columns
// [d * edoff, d * edoff + 32 KB) of the rows of E, produced step by step by a
// concurrently running bidirectional v6 backward recurrence (flag lines as
// X3PArgs streaming; the rows of step s are complete at epoch s + 3, the last
// step's at T + 2).  One persistent launch packs the rows as they appear
// (into Ap / eA) and runs the x3 GEMM tiles per direction; the two partials
// of a tile are added in a fixed order.  B_d packed along K (x3p_pack_cols).
struct X3PBwdStream {
  int M = 0, N = 0, KB = 0;            // frames (T * Nf), output columns, kb per direction
  const float *E = nullptr;
  long lde = 0, edoff = 0;
  _Float16 *Ap = nullptr;              // [2][M][KB][64]
  int *eA = nullptr;                   // [2][M]
  const _Float16 *B = nullptr;
  const int *eB = nullptr;
  long sB = 0, seB = 0;
  float *C = nullptr;
  long ldc = 0;
  float *part = nullptr;               // x3p_bwd_stream_part_floats(M, N) floats
  int *cnt = nullptr;                  // x3p_bwd_stream_ints(M, N) ints (zeroed here)
  const unsigned *flags = nullptr;     // producer flag lines
  int nwg = 0, T = 0, Nf = 0;
  int rg = 1;                          // producer row groups of 16 sequences
  unsigned *err = nullptr;
  int blocks = 0;                      // persistent blocks (each takes a CU: 96 KB LDS)
  bool bf16 = false;                   // rows packed as bf16 ([M][KB][64], KB 64-k blocks), B bf16, no exponents
  // XCD-pinned producer (rnn.hip xcd_mask): its workgroups OR
  // 1 << XCC_ID into *xcd_word as they start; a block waits until
  // xcd_count XCDs are registered and exits if it is on one of them
  const unsigned *xcd_word = nullptr;
  int xcd_count = 0;
  // FORWARD producer (the next component's input projection streamed off a
  // v6 forward's y rows, written through with the same epochs): direction 0
  // walks the frames upwards, 1 downwards; C += bias + bias2 of column c at
  // (c / bias_cols) * sbias + c % bias_cols.  256-tile launches only.
  float *part2 = nullptr;              // x3p_bwd_stream_part2_floats(N) floats (null: no split-K tail)
  int tail_rows = -1;                  // split-K tail slots per direction (-1: x3p_stream_tail_rows())
  bool forward = false;
  const float *bias = nullptr, *bias2 = nullptr;
  int bias_cols = 1;
  long sbias = 0;
};
size_t x3p_bwd_stream_ints(int M, int N);
// the launch runs on 256 x 256 tiles (512 threads, 128 KB LDS per block);
// part then needs x3p_bwd_stream_part_floats(M, N) floats
bool x3p_bwd_stream_256(int M, int N, int KB, bool bf16);
size_t x3p_bwd_stream_part_floats(int M, int N);
// split-K tail of the 256-tile launch (X3PBwdStream::part2): the last
// x3p_stream_tail_rows() row-tile slots of each direction, kStreamTailSplit ways
constexpr int kStreamTailSplit = 4;
int x3p_stream_tail_rows();
size_t x3p_bwd_stream_part2_floats(int N);
// test hook: the 256-tile row stream against a producer that has finished
// (every epoch final): C = sum_d pack(E[:, d K .. d K + K)) Wt_d^T (+ bias[c]),
// E [M][2K] row-major, Wt [2][N][K], device pointers; tail_rows as X3PBwdStream
void x3p_row_stream_selftest(hipStream_t s, int M, int N, int KB, int forward, int tail_rows, const float *E,
                             const float *Wt, const float *bias, float *C);
void gemm_x3p_bwd_stream(hipStream_t s, const X3PBwdStream &a);
// pack rows r < R of X (K values each, row stride ldx) -> out[b][r][KB][64],
// exponent per row into eout (bound > 0: from the bound, else the row max)
void x3p_pack_rows(hipStream_t s, const float *X, long ldx, int R, int K, _Float16 *out, int *eout, float bound,
                   int batch = 1, long sX = 0, long sOut = 0, long sE = 0);
// pack the transpose: packed row c < Cn = column c of X over its R rows
// (source row k - shift at k, zero outside), exponents from cmax[c] (float
// bits of max |x| of the column) or the bound
void x3p_pack_cols(hipStream_t s, const float *X, long ldx, int R, int Cn, int shift, _Float16 *out, int *eout,
                   const unsigned *cmax, float bound, int batch = 1, long sX = 0, long sOut = 0, long sE = 0,
                   long sCm = 0,
                   // avoid: X3PArgs::avoid_word; then counter: a zeroed int (dynamic item runs)
                   const unsigned *avoid = nullptr, int nxcd = 8, int *counter = nullptr);
inline size_t x3p_bytes(long rows, long K) { return (size_t)rows * ((K + 31) / 32) * 64 * 2; }

// column sums: out[b][j] (+)= alpha * sum_i X[b][i*ldx + j], i < rows  (accumulate if beta=1)
void colsum_f32(hipStream_t stream, const float *X, long ldx, int rows, int cols, float alpha,
                float beta, float *out, int batch = 1, long strideX = 0, long strideOut = 0);

}  // namespace kctc
