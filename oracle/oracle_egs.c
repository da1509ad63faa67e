/* oracle_egs.c -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's
 * cpu_baseline may load it; the product never does).  CPU restatement of
 * Kaldi's CompressedMatrix codec and of FormatNnetInput's packing, the
 * checker for kaldi-ctc_amd's egs path (host encoder, GPU decoder).
 *
 *   cm_* layout/arithmetic   src/matrix/compressed-matrix.h:128-171,
 *                            src/matrix/compressed-matrix.cc:27-38 (DataSize),
 *                            :41-123 (CopyFromMat), :193-210 (FloatToUint16 /
 *                            Uint16ToFloat), :212-291 (ComputeColHeader),
 *                            :293-335 (FloatToChar / CharToFloat), :438-481 (CopyToMat)
 *   oracle_format_input_cm   src/ctc/ctc-nnet-update.cc:351-424 (num_splice = 1)
 *
 * Built with -ffp-contract=off: the reference's arithmetic is a chain of
 * separately rounded float operations (x86-64 without FMA contraction), with
 * the integer-ramp terms of CharToFloat and the +0.5/+0.499 roundings in
 * double.  Parity: unpinned against the reference binary (no Kaldi build
 * here); pinned by the reference's own property tests
 * (src/matrix/matrix-lib-test.cc:4126-4297) in tests/test_egs.py. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int32_t format;
  float min_value, range;
  int32_t num_rows, num_cols;
} cm_hdr;

long oracle_cm_bytes(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  if (rows > 8) return 20 + (long)cols * (8 + rows);
  return 20 + 2L * rows * cols;
}

static uint16_t f2u16(const cm_hdr *h, float v) {
  float f = (v - h->min_value) / h->range;
  if (f > 1.0f) f = 1.0f;
  if (f < 0.0f) f = 0.0f;
  return (uint16_t)(int)(f * 65535 + 0.499);
}

static float u162f(const cm_hdr *h, uint16_t v) {
  return h->min_value + h->range * 1.52590218966964e-05F * v;
}

static unsigned char f2u8(float p0, float p25, float p75, float p100, float v) {
  int ans;
  if (v < p25) {
    float f = (v - p0) / (p25 - p0);
    ans = (int)(f * 64 + 0.5);
    if (ans < 0) ans = 0;
    if (ans > 64) ans = 64;
  } else if (v < p75) {
    float f = (v - p25) / (p75 - p25);
    ans = 64 + (int)(f * 128 + 0.5);
    if (ans < 64) ans = 64;
    if (ans > 192) ans = 192;
  } else {
    float f = (v - p75) / (p100 - p75);
    ans = 192 + (int)(f * 63 + 0.5);
    if (ans < 192) ans = 192;
    if (ans > 255) ans = 255;
  }
  return (unsigned char)ans;
}

static float u82f(float p0, float p25, float p75, float p100, unsigned char v) {
  if (v <= 64) return p0 + (p25 - p0) * v * (1 / 64.0);
  if (v <= 192) return p25 + (p75 - p25) * (v - 64) * (1 / 128.0);
  return p75 + (p100 - p75) * (v - 192) * (1 / 63.0);
}

static int cmpf(const void *a, const void *b) {
  float x = *(const float *)a, y = *(const float *)b;
  return (x > y) - (x < y);
}

static uint16_t umin(int a, int b) { return (uint16_t)(a < b ? a : b); }
static uint16_t umax(int a, int b) { return (uint16_t)(a > b ? a : b); }

/* returns bytes written (oracle_cm_bytes) or 0 for an empty matrix */
long oracle_cm_compress(const float *m, int rows, int cols, unsigned char *out) {
  if (rows <= 0 || cols <= 0) return 0;
  float mn = m[0], mx = m[0];
  for (long i = 0; i < (long)rows * cols; i++) {
    if (m[i] < mn) mn = m[i];
    if (m[i] > mx) mx = m[i];
  }
  if (mx == mn) mx = mn + (1.0 + fabs(mn));
  cm_hdr h;
  h.min_value = mn;
  h.range = mx - mn;
  if (h.range <= 0.0) h.range = 1.0e-05f;
  h.num_rows = rows;
  h.num_cols = cols;
  h.format = rows > 8 ? 1 : 2;
  memcpy(out, &h, 20);
  unsigned char *body = out + 20;
  if (h.format == 1) {
    unsigned char *bytes = body + 8L * cols;
    float *col = (float *)malloc(sizeof(float) * rows);
    for (int c = 0; c < cols; c++) {
      for (int r = 0; r < rows; r++) col[r] = m[(long)r * cols + c];
      qsort(col, rows, sizeof(float), cmpf);
      uint16_t p[4];
      if (rows >= 5) {
        int q = rows / 4;
        p[0] = umin(f2u16(&h, col[0]), 65532);
        p[1] = umin(umax(f2u16(&h, col[q]), p[0] + 1), 65533);
        p[2] = umin(umax(f2u16(&h, col[3 * q]), p[1] + 1), 65534);
        p[3] = umax(f2u16(&h, col[rows - 1]), p[2] + 1);
      } else {
        p[0] = umin(f2u16(&h, col[0]), 65532);
        p[1] = rows > 1 ? umin(umax(f2u16(&h, col[1]), p[0] + 1), 65533) : (uint16_t)(p[0] + 1);
        p[2] = rows > 2 ? umin(umax(f2u16(&h, col[2]), p[1] + 1), 65534) : (uint16_t)(p[1] + 1);
        p[3] = rows > 3 ? umax(f2u16(&h, col[3]), p[2] + 1) : (uint16_t)(p[2] + 1);
      }
      memcpy(body + 8L * c, p, 8);
      float p0 = u162f(&h, p[0]), p25 = u162f(&h, p[1]), p75 = u162f(&h, p[2]), p100 = u162f(&h, p[3]);
      for (int r = 0; r < rows; r++) bytes[(long)c * rows + r] = f2u8(p0, p25, p75, p100, m[(long)r * cols + c]);
    }
    free(col);
  } else {
    for (long i = 0; i < (long)rows * cols; i++) {
      uint16_t v = f2u16(&h, m[i]);
      memcpy(body + 2 * i, &v, 2);
    }
  }
  return oracle_cm_bytes(rows, cols);
}

/* data: GlobalHeader + body; out: rows x cols row-major */
void oracle_cm_decompress(const unsigned char *data, float *out) {
  cm_hdr h;
  memcpy(&h, data, 20);
  const unsigned char *body = data + 20;
  if (h.format == 1) {
    const unsigned char *bytes = body + 8L * h.num_cols;
    for (int c = 0; c < h.num_cols; c++) {
      uint16_t p[4];
      memcpy(p, body + 8L * c, 8);
      float p0 = u162f(&h, p[0]), p25 = u162f(&h, p[1]), p75 = u162f(&h, p[2]), p100 = u162f(&h, p[3]);
      for (int r = 0; r < h.num_rows; r++)
        out[(long)r * h.num_cols + c] = u82f(p0, p25, p75, p100, bytes[(long)c * h.num_rows + r]);
    }
  } else {
    for (long i = 0; i < (long)h.num_rows * h.num_cols; i++) {
      uint16_t v;
      memcpy(&v, body + 2 * i, 2);
      out[i] = u162f(&h, v);
    }
  }
}

/* FormatNnetInput, num_splice = 1: utterance n's decoded frames
 * [ignore, ignore + T_n) go to rows t*N + n (t < T_n) of out[T_max*N][dim+spk],
 * spk_info appended to every real frame, zero elsewhere.  images[n]: the
 * compressed image of utterance n, spk: [N][spk_dim]. */
void oracle_format_input_cm(const unsigned char *const *images, const int *ignore, const float *spk,
                            int spk_dim, int N, int T_max, float *out) {
  cm_hdr h0;
  memcpy(&h0, images[0], 20);
  const int Df = h0.num_cols, Dt = Df + spk_dim;
  memset(out, 0, sizeof(float) * (size_t)T_max * N * Dt);
  for (int n = 0; n < N; n++) {
    cm_hdr h;
    memcpy(&h, images[n], 20);
    float *m = (float *)malloc(sizeof(float) * (size_t)h.num_rows * h.num_cols);
    oracle_cm_decompress(images[n], m);
    const int Tn = h.num_rows - ignore[n];
    for (int t = 0; t < Tn && t < T_max; t++) {
      float *row = out + ((long)t * N + n) * Dt;
      memcpy(row, m + (long)(t + ignore[n]) * Df, sizeof(float) * Df);
      for (int j = 0; j < spk_dim; j++) row[Df + j] = spk[(long)n * spk_dim + j];
    }
    free(m);
  }
}
