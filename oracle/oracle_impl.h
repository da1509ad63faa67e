/*
 * oracle_impl.h -- body of the CPU restatement, instantiated twice by oracle.c
 * (REAL=double, SFX=_f64 and REAL=float, SFX=_f32).  TEST INFRASTRUCTURE ONLY
 * (see oracle.h for the parity status and who may load this code).
 */
#define FN(name) CAT(name, SFX)

/* ------------------------------------------------------------------------ */
/* GEMM: C[M][N] = alpha op(A) op(B) + beta C, row-major, blocked + OpenMP.  */
/* ------------------------------------------------------------------------ */
void FN(oracle_gemm)(int transA, int transB, int M, int N, int K, REAL alpha,
                     const REAL *A, int lda, const REAL *B, int ldb,
                     REAL beta, REAL *C, int ldc) {
  if (M <= 0 || N <= 0) return;
  /* materialise op(A) as [M][K] and op(B) as [K][N] row-major when transposed */
  const REAL *Ar = A, *Br = B;
  REAL *At = NULL, *Bt = NULL;
  int lda2 = lda, ldb2 = ldb;
  if (transA) {
    At = (REAL *)malloc(sizeof(REAL) * (size_t)M * (size_t)(K > 0 ? K : 1));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < M; i++)
      for (int k = 0; k < K; k++) At[(size_t)i * K + k] = A[(size_t)k * lda + i];
    Ar = At; lda2 = K;
  }
  if (transB) {
    Bt = (REAL *)malloc(sizeof(REAL) * (size_t)(K > 0 ? K : 1) * (size_t)N);
#pragma omp parallel for schedule(static)
    for (int k = 0; k < K; k++)
      for (int j = 0; j < N; j++) Bt[(size_t)k * N + j] = B[(size_t)j * ldb + k];
    Br = Bt; ldb2 = N;
  }
  /* tasks = (row block, column block) pairs so that the skinny per-step
   * recurrent GEMMs (M = minibatch) also spread over the threads */
  const int IB = 32, KB = 128, JB = M < 64 ? 64 : 512;
  const int nib = (M + IB - 1) / IB, njb = (N + JB - 1) / JB;
#pragma omp parallel for schedule(dynamic)
  for (int task = 0; task < nib * njb; task++) {
    const int ib = task / njb, jb = task - ib * njb;
    const int i0 = ib * IB, i1 = i0 + IB < M ? i0 + IB : M;
    const int j0 = jb * JB, j1 = j0 + JB < N ? j0 + JB : N, nj = j1 - j0;
    REAL acc[32 * 512];
    for (int i = i0; i < i1; i++)
      for (int j = 0; j < nj; j++) acc[(i - i0) * JB + j] = 0;
    for (int k0 = 0; k0 < K; k0 += KB) {
      int k1 = k0 + KB < K ? k0 + KB : K;
      for (int i = i0; i < i1; i++) {
        REAL *ci = acc + (i - i0) * JB;
        const REAL *ai = Ar + (size_t)i * lda2;
        for (int k = k0; k < k1; k++) {
          REAL a = ai[k];
          const REAL *bk = Br + (size_t)k * ldb2 + j0;
#pragma omp simd
          for (int j = 0; j < nj; j++) ci[j] += a * bk[j];
        }
      }
    }
    for (int i = i0; i < i1; i++) {
      REAL *ci = C + (size_t)i * ldc + j0;
      const REAL *ac = acc + (i - i0) * JB;
      if (beta == 0) {
        for (int j = 0; j < nj; j++) ci[j] = alpha * ac[j];
      } else {
        for (int j = 0; j < nj; j++) ci[j] = alpha * ac[j] + beta * ci[j];
      }
    }
  }
  free(At);
  free(Bt);
}

static REAL FN(lse2)(REAL a, REAL b) {
  if (a == (REAL)-INFINITY) return b;
  if (b == (REAL)-INFINITY) return a;
  REAL m = a > b ? a : b;
  return m + (REAL)log1p(exp((a > b ? b - a : a - b)));
}

/* ------------------------------------------------------------------------ */
/* CTC: warp-ctc compute_ctc_loss semantics (called from                     */
/* src/ctc/ctc-nnet-update.cc:211-243; blank_label = 0 at :205).             */
/* ------------------------------------------------------------------------ */
void FN(oracle_ctc)(const REAL *acts, REAL *grads, const int *flat_labels,
                    const int *label_lengths, const int *input_lengths,
                    int A, int N, int T_max, REAL *costs, int blank) {
  int *offs = (int *)malloc(sizeof(int) * (N + 1));
  offs[0] = 0;
  for (int n = 0; n < N; n++) offs[n + 1] = offs[n] + label_lengths[n];
  if (grads) {
    /* rows t >= T_n (zero padding of FormatNnetInput) get a zero gradient:
     * the reference pre-zeroes the gradient matrix (ctc-nnet-update.cc:222) */
    for (size_t i = 0; i < (size_t)T_max * N * A; i++) grads[i] = 0;
  }
#pragma omp parallel for schedule(dynamic)
  for (int n = 0; n < N; n++) {
    const int T = input_lengths[n], L = label_lengths[n], S = 2 * L + 1;
    const int *lab = flat_labels + offs[n];
    int repeats = 0;
    for (int i = 1; i < L; i++) repeats += (lab[i] == lab[i - 1]);
    if (T <= 0 || L + repeats > T) { costs[n] = 0; continue; }
    int *ext = (int *)malloc(sizeof(int) * S);
    for (int s = 0; s < S; s++) ext[s] = (s & 1) ? lab[(s - 1) / 2] : blank;
    REAL *logy = (REAL *)malloc(sizeof(REAL) * (size_t)T * A);
    for (int t = 0; t < T; t++) {
      const REAL *row = acts + ((size_t)t * N + n) * A;
      REAL m = row[0];
      for (int a = 1; a < A; a++) m = row[a] > m ? row[a] : m;
      REAL z = 0;
      for (int a = 0; a < A; a++) z += (REAL)exp(row[a] - m);
      REAL lz = m + (REAL)log(z);
      for (int a = 0; a < A; a++) logy[(size_t)t * A + a] = row[a] - lz;
    }
    REAL *alpha = (REAL *)malloc(sizeof(REAL) * (size_t)T * S);
    REAL *beta = (REAL *)malloc(sizeof(REAL) * (size_t)T * S);
    for (size_t i = 0; i < (size_t)T * S; i++) alpha[i] = beta[i] = (REAL)-INFINITY;
    alpha[0] = logy[ext[0]];
    if (S > 1) alpha[1] = logy[ext[1]];
    for (int t = 1; t < T; t++) {
      const REAL *ap = alpha + (size_t)(t - 1) * S;
      REAL *ac = alpha + (size_t)t * S;
      for (int s = 0; s < S; s++) {
        REAL v = ap[s];
        if (s >= 1) v = FN(lse2)(v, ap[s - 1]);
        if (s >= 2 && ext[s] != blank && ext[s] != ext[s - 2]) v = FN(lse2)(v, ap[s - 2]);
        ac[s] = (v == (REAL)-INFINITY) ? v : v + logy[(size_t)t * A + ext[s]];
      }
    }
    const REAL *al = alpha + (size_t)(T - 1) * S;
    REAL logp = al[S - 1];
    if (S > 1) logp = FN(lse2)(logp, al[S - 2]);
    costs[n] = -logp;
    if (grads) {
      /* beta_t(s): probability of finishing from state s at t, EXCLUDING
       * the emission at t, so that alpha_t(s) beta_t(s) = P(s at t). */
      REAL *bl = beta + (size_t)(T - 1) * S;
      bl[S - 1] = 0;
      if (S > 1) bl[S - 2] = 0;
      for (int t = T - 2; t >= 0; t--) {
        const REAL *bn = beta + (size_t)(t + 1) * S;
        const REAL *ly = logy + (size_t)(t + 1) * A;
        REAL *bc = beta + (size_t)t * S;
        for (int s = 0; s < S; s++) {
          REAL v = bn[s] + ly[ext[s]];
          if (s + 1 < S) v = FN(lse2)(v, bn[s + 1] + ly[ext[s + 1]]);
          if (s + 2 < S && ext[s + 2] != blank && ext[s + 2] != ext[s])
            v = FN(lse2)(v, bn[s + 2] + ly[ext[s + 2]]);
          bc[s] = v;
        }
      }
      REAL *gam = (REAL *)malloc(sizeof(REAL) * A);
      for (int t = 0; t < T; t++) {
        for (int a = 0; a < A; a++) gam[a] = 0;
        for (int s = 0; s < S; s++) {
          REAL v = alpha[(size_t)t * S + s] + beta[(size_t)t * S + s];
          if (v != (REAL)-INFINITY) gam[ext[s]] += (REAL)exp(v - logp);
        }
        REAL *g = grads + ((size_t)t * N + n) * A;
        for (int a = 0; a < A; a++) g[a] = (REAL)exp(logy[(size_t)t * A + a]) - gam[a];
      }
      free(gam);
    }
    free(ext); free(logy); free(alpha); free(beta);
  }
  free(offs);
}

/* ------------------------------------------------------------------------ */
/* cuDNN-v5 style recurrent layer                                            */
/* ------------------------------------------------------------------------ */
static REAL FN(sigm)(REAL x) { return (REAL)1 / ((REAL)1 + (REAL)exp(-x)); }
static REAL FN(act)(int mode, REAL x) {
  return mode == ORACLE_RNN_RELU ? (x > 0 ? x : 0) : (REAL)tanh(x);
}

/* One stacked layer, both directions.  wbase = params of pseudo-layer
 * (layer*dirs + 0); the next direction's block follows contiguously. */
static void FN(rnn_layer_fwd)(int mode, int T, int N, int Din, int H, int dirs,
                              const REAL *x, const REAL *params, int D0, int layers,
                              int layer, REAL *y, REAL *res) {
  const int nW = oracle_nw(mode), ns = oracle_ns(mode), G4 = nW * H;
  const size_t TN = (size_t)T * N;
  REAL *G = (REAL *)malloc(sizeof(REAL) * TN * G4);
  REAL *Rh = (REAL *)malloc(sizeof(REAL) * (size_t)N * G4);
  REAL *c = (REAL *)malloc(sizeof(REAL) * (size_t)N * H);
  REAL *Rt = (REAL *)malloc(sizeof(REAL) * (size_t)H * G4);
  for (int d = 0; d < dirs; d++) {
    int p = layer * dirs + d;
    const REAL *W = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, 0, 0);
    const REAL *R = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, nW, 0);
    for (int j = 0; j < G4; j++)  /* R^T once per direction: the per-step GEMM is then NN */
      for (int k = 0; k < H; k++) Rt[(size_t)k * G4 + j] = R[(size_t)j * H + k];
    const REAL *bW = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, 0, 1);
    const REAL *bR = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, nW, 1);
    FN(oracle_gemm)(0, 1, (int)TN, G4, Din, 1, x, Din, W, Din, 0, G, G4);
    for (size_t r = 0; r < TN; r++)
      for (int j = 0; j < G4; j++) G[r * G4 + j] += bW[j];
    for (int i = 0; i < N * H; i++) c[i] = 0;
    for (int k = 0; k < T; k++) {
      int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
      const int ldy = dirs * H;
      if (k == 0) {
        for (int n = 0; n < N; n++)
          for (int j = 0; j < G4; j++) Rh[n * G4 + j] = bR[j];
      } else {
        for (int n = 0; n < N; n++)
          for (int j = 0; j < G4; j++) Rh[n * G4 + j] = bR[j];
        FN(oracle_gemm)(0, 0, N, G4, H, 1, y + (size_t)tp * N * ldy + d * H, ldy, Rt, G4, 1, Rh, G4);
      }
      for (int n = 0; n < N; n++) {
        const REAL *g = G + ((size_t)t * N + n) * G4;
        const REAL *rh = Rh + (size_t)n * G4;
        REAL *st = res + (((size_t)t * N + n) * dirs + d) * (size_t)ns * H;
        REAL *yo = y + ((size_t)t * N + n) * ldy + d * H;
        const REAL *hp = k == 0 ? NULL : y + ((size_t)tp * N + n) * ldy + d * H;
        for (int j = 0; j < H; j++) {
          if (mode == ORACLE_RNN_LSTM) {
            REAL ig = FN(sigm)(g[j] + rh[j]);
            REAL fg = FN(sigm)(g[H + j] + rh[H + j]);
            REAL gg = (REAL)tanh(g[2 * H + j] + rh[2 * H + j]);
            REAL og = FN(sigm)(g[3 * H + j] + rh[3 * H + j]);
            REAL cc = fg * c[n * H + j] + ig * gg;
            c[n * H + j] = cc;
            st[j] = ig; st[H + j] = fg; st[2 * H + j] = gg; st[3 * H + j] = og; st[4 * H + j] = cc;
            yo[j] = og * (REAL)tanh(cc);
          } else if (mode == ORACLE_RNN_GRU) {
            REAL r = FN(sigm)(g[j] + rh[j]);
            REAL z = FN(sigm)(g[H + j] + rh[H + j]);
            REAL nn = (REAL)tanh(g[2 * H + j] + r * rh[2 * H + j]);
            REAL h0 = hp ? hp[j] : 0;
            st[j] = r; st[H + j] = z; st[2 * H + j] = nn; st[3 * H + j] = rh[2 * H + j];
            yo[j] = (1 - z) * nn + z * h0;
          } else {
            REAL h = FN(act)(mode, g[j] + rh[j]);
            st[j] = h;
            yo[j] = h;
          }
        }
      }
    }
  }
  free(G); free(Rh); free(c); free(Rt);
}

static void FN(rnn_layer_bwd)(int mode, int T, int N, int Din, int H, int dirs,
                              const REAL *x, const REAL *params, int D0, int layers,
                              int layer, const REAL *y, const REAL *dy, const REAL *res,
                              REAL *dx, REAL *dw) {
  const int nW = oracle_nw(mode), ns = oracle_ns(mode), G4 = nW * H, ldy = dirs * H;
  const size_t TN = (size_t)T * N;
  REAL *DPX = (REAL *)malloc(sizeof(REAL) * TN * G4);
  REAL *DPH = (REAL *)malloc(sizeof(REAL) * TN * G4);
  REAL *HP = (REAL *)malloc(sizeof(REAL) * TN * H);
  REAL *dhrec = (REAL *)malloc(sizeof(REAL) * (size_t)N * H);
  REAL *dcc = (REAL *)malloc(sizeof(REAL) * (size_t)N * H);
  if (dx)
    for (size_t i = 0; i < TN * Din; i++) dx[i] = 0;
  for (int d = 0; d < dirs; d++) {
    int p = layer * dirs + d;
    const REAL *W = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, 0, 0);
    const REAL *R = params + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, nW, 0);
    for (int i = 0; i < N * H; i++) dhrec[i] = dcc[i] = 0;
    for (int k = T - 1; k >= 0; k--) {
      int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
      for (int n = 0; n < N; n++) {
        const REAL *st = res + (((size_t)t * N + n) * dirs + d) * (size_t)ns * H;
        const REAL *stp = k == 0 ? NULL : res + (((size_t)tp * N + n) * dirs + d) * (size_t)ns * H;
        const REAL *hp = k == 0 ? NULL : y + ((size_t)tp * N + n) * ldy + d * H;
        const REAL *hh = y + ((size_t)t * N + n) * ldy + d * H;
        const REAL *dyo = dy + ((size_t)t * N + n) * ldy + d * H;
        REAL *dpx = DPX + ((size_t)t * N + n) * G4;
        REAL *dph = DPH + ((size_t)t * N + n) * G4;
        REAL *hpo = HP + ((size_t)t * N + n) * H;
        for (int j = 0; j < H; j++) {
          REAL dh = dyo[j] + dhrec[n * H + j];
          hpo[j] = hp ? hp[j] : 0;
          if (mode == ORACLE_RNN_LSTM) {
            REAL ig = st[j], fg = st[H + j], gg = st[2 * H + j], og = st[3 * H + j], cc = st[4 * H + j];
            REAL cp = stp ? stp[4 * H + j] : 0;
            REAL tc = (REAL)tanh(cc);
            REAL dO = dh * tc;
            REAL dc = dh * og * (1 - tc * tc) + dcc[n * H + j];
            REAL dI = dc * gg, dG = dc * ig, dF = dc * cp;
            dcc[n * H + j] = dc * fg;
            dpx[j] = dph[j] = dI * ig * (1 - ig);
            dpx[H + j] = dph[H + j] = dF * fg * (1 - fg);
            dpx[2 * H + j] = dph[2 * H + j] = dG * (1 - gg * gg);
            dpx[3 * H + j] = dph[3 * H + j] = dO * og * (1 - og);
          } else if (mode == ORACLE_RNN_GRU) {
            REAL r = st[j], z = st[H + j], nn = st[2 * H + j], rhn = st[3 * H + j];
            REAL h0 = hp ? hp[j] : 0;
            REAL dn = dh * (1 - z), dz = dh * (h0 - nn);
            REAL dpn = dn * (1 - nn * nn);
            REAL dpr = dpn * rhn * r * (1 - r);
            REAL dpz = dz * z * (1 - z);
            dpx[j] = dph[j] = dpr;
            dpx[H + j] = dph[H + j] = dpz;
            dpx[2 * H + j] = dpn;
            dph[2 * H + j] = dpn * r;
            dcc[n * H + j] = dh * z; /* direct path to h_{prev} */
          } else {
            REAL h = hh[j];
            REAL der = mode == ORACLE_RNN_RELU ? (h > 0 ? 1 : 0) : (1 - h * h);
            dpx[j] = dph[j] = dh * der;
          }
        }
      }
      /* dh_rec for the step processed next (previous in forward order) */
      FN(oracle_gemm)(0, 0, N, H, G4, 1, DPH + (size_t)t * N * G4, G4, R, H, 0, dhrec, H);
      if (mode == ORACLE_RNN_GRU)
        for (int i = 0; i < N * H; i++) dhrec[i] += dcc[i];
    }
    if (dx) FN(oracle_gemm)(0, 0, (int)TN, Din, G4, 1, DPX, G4, W, Din, 1, dx, Din);
    if (dw) {
      REAL *dW = dw + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, 0, 0);
      REAL *dR = dw + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, nW, 0);
      REAL *dbW = dw + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, 0, 1);
      REAL *dbR = dw + oracle_rnn_lin_offset(mode, D0, H, layers, dirs, p, nW, 1);
      FN(oracle_gemm)(1, 0, G4, Din, (int)TN, 1, DPX, G4, x, Din, 1, dW, Din);
      FN(oracle_gemm)(1, 0, G4, H, (int)TN, 1, DPH, G4, HP, H, 1, dR, H);
      for (int j = 0; j < G4; j++) {
        REAL sx = 0, sh = 0;
        for (size_t r = 0; r < TN; r++) { sx += DPX[r * G4 + j]; sh += DPH[r * G4 + j]; }
        dbW[j] += sx;
        dbR[j] += sh;
      }
    }
  }
  free(DPX); free(DPH); free(HP); free(dhrec); free(dcc);
}

void FN(oracle_rnn_forward)(int mode, int T, int N, int D, int H, int layers, int dirs,
                            const REAL *x, const REAL *w, REAL *y, REAL *reserve) {
  const int ns = oracle_ns(mode);
  const size_t per_state = (size_t)T * N * dirs * ns * H, per_out = (size_t)T * N * dirs * H;
  REAL *outs = reserve + per_state * layers;
  const REAL *in = x;
  for (int l = 0; l < layers; l++) {
    REAL *out = (l == layers - 1) ? y : outs + per_out * l;
    FN(rnn_layer_fwd)(mode, T, N, l == 0 ? D : dirs * H, H, dirs, in, w, D, layers, l, out,
                      reserve + per_state * l);
    in = out;
  }
}

void FN(oracle_rnn_backward)(int mode, int T, int N, int D, int H, int layers, int dirs,
                             const REAL *x, const REAL *w, const REAL *y, const REAL *dy,
                             const REAL *reserve, REAL *dx, REAL *dw) {
  const int ns = oracle_ns(mode);
  const size_t per_state = (size_t)T * N * dirs * ns * H, per_out = (size_t)T * N * dirs * H;
  const REAL *outs = reserve + per_state * layers;
  REAL *dcur = (REAL *)malloc(sizeof(REAL) * per_out);
  REAL *dnext = (REAL *)malloc(sizeof(REAL) * per_out);
  memcpy(dcur, dy, sizeof(REAL) * per_out);
  for (int l = layers - 1; l >= 0; l--) {
    const REAL *in = l == 0 ? x : outs + per_out * (l - 1);
    const REAL *out = l == layers - 1 ? y : outs + per_out * l;
    REAL *dxl = l == 0 ? dx : dnext;
    FN(rnn_layer_bwd)(mode, T, N, l == 0 ? D : dirs * H, H, dirs, in, w, D, layers, l, out,
                      dcur, reserve + per_state * l, dxl, dw);
    if (l > 0) { REAL *tmp = dcur; dcur = dnext; dnext = tmp; }
  }
  free(dcur); free(dnext);
}

/* ------------------------------------------------------------------------ */
/* Whole train step (NnetCtcUpdater::ComputeForMinibatch with SGD update).   */
/* ------------------------------------------------------------------------ */
/* ClipGradientComponent::Backprop + RepairGradients, norm-based
 * (src/nnet2/nnet-cudnn-component.cc:921-1055).  d [rows][dim] in place. */
static void FN(clip_gradient_bwd)(const oracle_nnet_spec *sp, const REAL *in_value,
                                  REAL *d, long rows, int dim, float draw,
                                  double *num_clipped, double *count) {
  const double thr = sp->clip_threshold;
  if (thr <= 0) return;
  long not_scaled = 0;
  for (long r = 0; r < rows; r++) {
    REAL *row = d + r * dim;
    REAL ss = 0;
    for (int j = 0; j < dim; j++) ss += row[j] * row[j];
    REAL sc = ss * (REAL)(1.0 / (thr * thr));
    if (sc < 1) { not_scaled++; continue; }
    REAL f = (REAL)(1.0 / sqrt((double)sc));
    for (int j = 0; j < dim; j++) row[j] *= f;
  }
  *num_clipped += (double)(rows - not_scaled);
  *count += (double)rows;
  /* RepairGradients (:980-1055); repair_probability 0.5 */
  if (sp->repair_threshold >= 1.0 || sp->repair_scale == 0 || *count == 0 || draw > 0.5f) return;
  double prop = *num_clipped / *count;
  if (prop <= sp->repair_threshold) return;
  REAL *rep = (REAL *)malloc(sizeof(REAL) * rows * dim);
  for (long i = 0; i < rows * dim; i++) {
    REAL v = in_value[i];
    REAL sgn = v > 0 ? 1 : -1;
    REAL m = (REAL)fabs((double)v) - (REAL)sp->repair_target;
    rep[i] = (m > 0 ? m : 0) * sgn;
  }
  double dn = 0, rn = 0;
  for (long r = 0; r < rows; r++) {
    REAL a = 0, b = 0;
    for (int j = 0; j < dim; j++) { a += d[r * dim + j] * d[r * dim + j]; b += rep[r * dim + j] * rep[r * dim + j]; }
    dn += sqrt((double)a); rn += sqrt((double)b);
  }
  double magnitude = sp->repair_scale * prop * (dn / rows);
  double scale = rn != 0 ? magnitude / (rn / rows) : 0;
  REAL alpha = (REAL)(-scale / 0.5);
  for (long i = 0; i < rows * dim; i++) d[i] += alpha * rep[i];
  double dn2 = 0;
  for (long r = 0; r < rows; r++) {
    REAL a = 0;
    for (int j = 0; j < dim; j++) a += d[r * dim + j] * d[r * dim + j];
    dn2 += sqrt((double)a);
  }
  if (dn2 != 0) {
    REAL f = (REAL)(dn / dn2);
    for (long i = 0; i < rows * dim; i++) d[i] *= f;
  }
  free(rep);
}

double FN(oracle_train_step)(const oracle_nnet_spec *sp, REAL **rnn_params,
                             REAL *affine_W, REAL *affine_b, const REAL *feats,
                             int T, int N, const int *num_frames, const int *flat_labels,
                             const int *label_lengths, const float *repair_draws,
                             double *clip_num_clipped, double *clip_count,
                             double *tot_accuracy, double *tot_weight) {
  return FN(oracle_train_step_ex)(sp, rnn_params, affine_W, affine_b, feats, T, N, num_frames, flat_labels,
                                  label_lengths, repair_draws, clip_num_clipped, clip_count, tot_accuracy,
                                  tot_weight, NULL, NULL, NULL);
}

double FN(oracle_train_step_ex)(const oracle_nnet_spec *sp, REAL **rnn_params,
                                REAL *affine_W, REAL *affine_b, const REAL *feats,
                                int T, int N, const int *num_frames, const int *flat_labels,
                                const int *label_lengths, const float *repair_draws,
                                double *clip_num_clipped, double *clip_count,
                                double *tot_accuracy, double *tot_weight,
                                double *costs_out, REAL *logits_out, int *ids_out) {
  const int C = sp->num_rnn, H = sp->hidden, dirs = sp->dirs, Lr = sp->layers_per_rnn;
  const int A = sp->num_targets, Dout = dirs * H, mode = sp->mode;
  const long rows = (long)T * N;
  REAL **ys = (REAL **)malloc(sizeof(REAL *) * C);
  REAL **res = (REAL **)malloc(sizeof(REAL *) * C);
  const REAL *in = feats;
  for (int c = 0; c < C; c++) {
    int Din = c == 0 ? sp->input_dim : Dout;
    ys[c] = (REAL *)malloc(sizeof(REAL) * rows * Dout);
    res[c] = (REAL *)malloc(sizeof(REAL) * oracle_rnn_reserve_size(mode, T, N, H, Lr, dirs));
    FN(oracle_rnn_forward)(mode, T, N, Din, H, Lr, dirs, in, rnn_params[c], ys[c], res[c]);
    in = ys[c];  /* ClipGradientComponent::Propagate is a copy */
  }
  REAL *logits = (REAL *)malloc(sizeof(REAL) * rows * A);
  for (long r = 0; r < rows; r++)
    for (int a = 0; a < A; a++) logits[r * A + a] = affine_b[a];
  FN(oracle_gemm)(0, 1, (int)rows, A, Dout, 1, in, Dout, affine_W, Dout, 1, logits, A);
  REAL *grad = (REAL *)malloc(sizeof(REAL) * rows * A);
  REAL *costs = (REAL *)malloc(sizeof(REAL) * N);
  FN(oracle_ctc)(logits, grad, flat_labels, label_lengths, num_frames, A, N, T, costs, 0);
  double tot = 0;
  for (int n = 0; n < N; n++) tot += costs[n];
  if (costs_out)
    for (int n = 0; n < N; n++) costs_out[n] = (double)costs[n];
  if (logits_out) memcpy(logits_out, logits, sizeof(REAL) * rows * A);
  /* accuracy on the forward logits, best path by the GPU _find_row_max_id
   * rule (oracle_find_row_max_id_f32; cu-kernels.cu:2454-2500) in REAL */
  {
    int *ids = (int *)malloc(sizeof(int) * rows);
    REAL smax[256];
    int sidx[256];
    for (long r = 0; r < rows; r++) {
      for (int t = 0; t < 256; t++) {
        REAL tmax = (REAL)-1e20f;
        int tidx = -1;
        for (int a = t; a < A; a += 256)
          if (logits[r * A + a] > tmax) { tmax = logits[r * A + a]; tidx = a; }
        smax[t] = tmax;
        sidx[t] = tidx;
      }
      for (int w = 128; w >= 1; w >>= 1)
        for (int p = 0; p < w; p++)
          if (smax[p + w] > smax[p]) { smax[p] = smax[p + w]; sidx[p] = sidx[p + w]; }
      ids[r] = sidx[0];
    }
    *tot_accuracy = oracle_ctc_accuracy(ids, T, N, num_frames, flat_labels, label_lengths, tot_weight);
    if (ids_out) memcpy(ids_out, ids, sizeof(int) * rows);
    free(ids);
  }
  /* Backprop: deriv *= -1 (ctc-nnet-update.cc:323) */
  for (long i = 0; i < rows * A; i++) grad[i] = -grad[i];
  REAL *dx = (REAL *)malloc(sizeof(REAL) * rows * Dout);
  FN(oracle_gemm)(0, 0, (int)rows, Dout, A, 1, grad, A, affine_W, Dout, 0, dx, Dout);
  for (int a = 0; a < A; a++) {
    REAL s = 0;
    for (long r = 0; r < rows; r++) s += grad[r * A + a];
    affine_b[a] += (REAL)sp->lr_affine * s;
  }
  FN(oracle_gemm)(1, 0, A, Dout, (int)rows, (REAL)sp->lr_affine, grad, A, in, Dout, 1, affine_W, Dout);
  REAL *dnext = (REAL *)malloc(sizeof(REAL) * rows * (sp->input_dim > Dout ? sp->input_dim : Dout));
  for (int c = C - 1; c >= 0; c--) {
    int Din = c == 0 ? sp->input_dim : Dout;
    FN(clip_gradient_bwd)(sp, ys[c], dx, rows, Dout, repair_draws ? repair_draws[c] : 1.0f,
                          &clip_num_clipped[c], &clip_count[c]);
    long P = oracle_rnn_params_size(mode, Din, H, Lr, dirs);
    REAL *dw = (REAL *)calloc((size_t)P, sizeof(REAL));
    const REAL *xin = c == 0 ? feats : ys[c - 1];
    FN(oracle_rnn_backward)(mode, T, N, Din, H, Lr, dirs, xin, rnn_params[c], ys[c], dx, res[c],
                            c == 0 ? NULL : dnext, dw);
    const REAL cg = (REAL)sp->rnn_clip_gradient;
    for (long i = 0; i < P; i++) {
      REAL g = dw[i];
      if (g < -cg) g = -cg;
      if (g > cg) g = cg;
      rnn_params[c][i] += (REAL)sp->lr_rnn * g;
    }
    free(dw);
    if (c > 0) { REAL *t = dx; dx = dnext; dnext = t; }
  }
  for (int c = 0; c < C; c++) { free(ys[c]); free(res[c]); }
  free(ys); free(res); free(logits); free(grad); free(costs); free(dx); free(dnext);
  return tot;
}

#undef FN
