/*
 * oracle.c -- CPU restatement of the kaldi-ctc CTC-training hot path.
 * TEST INFRASTRUCTURE ONLY; see oracle.h for scope and parity status
 * ("parity unpinned" against the reference; cross-checked against torch fp64
 * through tests/golden/).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle.h"

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)

/* number of input-weight matrices per pseudo-layer (= gates) */
static int oracle_nw(int mode) {
  return mode == ORACLE_RNN_LSTM ? 4 : mode == ORACLE_RNN_GRU ? 3 : 1;
}
/* floats of per-(t,n,dir) state kept for backward, in units of H */
static int oracle_ns(int mode) {
  return mode == ORACLE_RNN_LSTM ? 5 : mode == ORACLE_RNN_GRU ? 4 : 1;
}

static long pl_size(int mode, int Din, int H) {
  long nW = oracle_nw(mode);
  return nW * H * (long)Din + nW * H * (long)H + 2 * nW * H;
}

long oracle_rnn_params_size(int mode, int D, int H, int layers, int dirs) {
  long tot = 0;
  for (int l = 0; l < layers; l++)
    tot += dirs * pl_size(mode, l == 0 ? D : dirs * H, H);
  return tot;
}

long oracle_rnn_lin_offset(int mode, int D, int H, int layers, int dirs,
                           int pseudo_layer, int lin_id, int is_bias) {
  (void)layers;
  long off = 0;
  int layer = pseudo_layer / dirs;
  for (int p = 0; p < pseudo_layer; p++) off += pl_size(mode, (p / dirs) == 0 ? D : dirs * H, H);
  int Din = layer == 0 ? D : dirs * H;
  long nW = oracle_nw(mode);
  if (!is_bias) {
    if (lin_id < nW) return off + (long)lin_id * H * Din;
    return off + nW * H * (long)Din + (long)(lin_id - nW) * H * H;
  }
  return off + nW * H * (long)Din + nW * H * (long)H + (long)lin_id * H;
}

long oracle_rnn_reserve_size(int mode, int T, int N, int H, int layers, int dirs) {
  long st = (long)T * N * dirs * oracle_ns(mode) * H * layers;
  long outs = (long)T * N * dirs * H * (layers > 1 ? layers - 1 : 0);
  return st + outs;
}

int oracle_levenshtein(const int *a, int na, const int *b, int nb) {
  /* LevenshteinEditDistance (src/util/edit-distance-inl.h): unit costs */
  int *prev = (int *)malloc(sizeof(int) * (nb + 1));
  int *cur = (int *)malloc(sizeof(int) * (nb + 1));
  for (int j = 0; j <= nb; j++) prev[j] = j;
  for (int i = 1; i <= na; i++) {
    cur[0] = i;
    for (int j = 1; j <= nb; j++) {
      int sub = prev[j - 1] + (a[i - 1] != b[j - 1]);
      int del = prev[j] + 1, ins = cur[j - 1] + 1;
      int m = sub < del ? sub : del;
      cur[j] = m < ins ? m : ins;
    }
    int *t = prev; prev = cur; cur = t;
  }
  int r = prev[nb];
  free(prev); free(cur);
  return r;
}

/* CPU CuMatrixBase::FindRowMaxId (src/cudamatrix/cu-matrix.cc:1630-1644):
 * first strict maximum above -1e21, -1 when there is none. */
void oracle_find_row_max_id_cpu_f32(const float *m, int rows, int cols, int *ids) {
  for (int r = 0; r < rows; r++) {
    const float *row = m + (size_t)r * cols;
    float mx = -1e21f;
    int b = -1;
    for (int c = 0; c < cols; c++)
      if (mx < row[c]) { mx = row[c]; b = c; }
    ids[r] = b;
  }
}

/* GPU _find_row_max_id (src/cudamatrix/cu-kernels.cu:2454-2500), the kernel
 * the reference's CTC path runs (CTC_GPU is hard-wired, ComputeTotAccuracy ->
 * FindRowMaxId on a device matrix, src/ctc/ctc-nnet-update.cc:270-273):
 * block of CU1DBLOCK = 256 threads per row; thread t keeps the first strict
 * maximum above -1e20f of columns t, t+256, ... (index -1 if none), then a
 * shared-memory tree halves the active threads (128, 64, 32 with barriers,
 * then 16 .. 1 inside one warp) and position p takes position p+w only when
 * strictly greater.  Ties between threads therefore resolve by the tree, not
 * to the lowest column: equal maxima at columns 1 and 2 give 2.  Rows whose
 * values are all <= -1e20 (or NaN) give -1. */
void oracle_find_row_max_id_f32(const float *m, int rows, int cols, int *ids) {
  enum { B = 256 };
  float smax[B];
  int sidx[B];
  for (int r = 0; r < rows; r++) {
    const float *row = m + (size_t)r * cols;
    for (int t = 0; t < B; t++) {
      float tmax = -1e20f;
      int tidx = -1;
      for (int j = t; j < cols; j += B)
        if (row[j] > tmax) { tmax = row[j]; tidx = j; }
      smax[t] = tmax;
      sidx[t] = tidx;
    }
    /* within one level reads (p + w >= w) and writes (p < w) are disjoint */
    for (int w = B / 2; w >= 1; w >>= 1)
      for (int p = 0; p < w; p++)
        if (smax[p + w] > smax[p]) { smax[p] = smax[p + w]; sidx[p] = sidx[p + w]; }
    ids[r] = sidx[0];
  }
}

/* SoftmaxComponent::Propagate (src/nnet2/nnet-component.cc:929-946): per row
 * exp(x - max) / sum, floored at 1e-20 (computed in double, rounded once). */
void oracle_softmax_rows_f32(const float *in, long rows, int cols, float *out) {
  for (long r = 0; r < rows; r++) {
    const float *x = in + r * cols;
    double m = x[0], s = 0;
    for (int j = 1; j < cols; j++) m = x[j] > m ? x[j] : m;
    for (int j = 0; j < cols; j++) s += exp((double)x[j] - m);
    for (int j = 0; j < cols; j++) {
      double v = exp((double)x[j] - m) / s;
      out[r * cols + j] = (float)(v > 1e-20 ? v : 1e-20);
    }
  }
}

/* CtcDecodableAmNnet (src/ctc/ctc-decodable-am-nnet.cc:28-80) on the network
 * output probs [T][A]: blank-threshold frame skip (probs[t][0] <
 * blank_threshold keeps t; none kept -> all kept), ApplyFloor(floor_v),
 * ApplyLog, AddVecToRows(-1, log(priors)) when priors, Scale(prob_scale).
 * Returns the number of rows written to out. */
int oracle_ctc_decodable_f32(const float *probs, int T, int A, const float *priors, float prob_scale,
                             float blank_threshold, float floor_v, float *out) {
  int kept = 0;
  for (int pass = 0; pass < 2 && kept == 0; pass++) {
    const int skip = pass == 0 && blank_threshold < 1.0f;
    kept = 0;
    for (int t = 0; t < T; t++) {
      if (skip && !(probs[(long)t * A] < blank_threshold)) continue;
      for (int a = 0; a < A; a++) {
        float p = probs[(long)t * A + a];
        float v = logf(p > floor_v ? p : floor_v);
        if (priors) v += -1.0f * logf(priors[a]);
        out[(long)kept * A + a] = v * prob_scale;
      }
      kept++;
    }
    if (!skip) break;
  }
  return kept;
}

double oracle_ctc_accuracy(const int *best_ids, int T_max, int N,
                           const int *num_frames, const int *flat_labels,
                           const int *label_lengths, double *tot_weight) {
  (void)T_max;
  const int blank = 0;
  double tot_num = 0, err = 0;
  int off = 0;
  int *hyp = (int *)malloc(sizeof(int) * (T_max > 0 ? T_max : 1));
  for (int n = 0; n < N; n++) {
    int F = num_frames[n], L = label_lengths[n];
    tot_num += L;
    for (int i = 0; i < F; i++) hyp[i] = best_ids[(size_t)i * N + n];
    /* collapse: loop from i = j = 1, hyp[0] always kept (:291-303) */
    int i = 1, j = 1;
    while (j < F) {
      if (hyp[j] != hyp[j - 1] && hyp[j] != blank) { hyp[i] = hyp[j]; i++; }
      j++;
    }
    int nh = F > 0 ? i : 0;
    err += oracle_levenshtein(flat_labels + off, L, hyp, nh);
    off += L;
  }
  free(hyp);
  if (tot_weight) *tot_weight = tot_num;
  return tot_num - err;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

#define REAL double
#define SFX _f64
#include "oracle_impl.h"
#undef REAL
#undef SFX

#define REAL float
#define SFX _f32
#include "oracle_impl.h"
#undef REAL
#undef SFX
