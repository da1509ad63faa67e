/*
 * oracle.h -- CPU restatement of the kaldi-ctc CTC-training hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so -- as the checker, never
 * as the thing measured or shipped.  The product (kaldi-ctc_amd/) never links
 * or calls anything in this directory.
 *
 * Parity status: the reference's arithmetic lives in two third-party libraries
 * that are NOT in /root/reference (warp-ctc, lifeiteng fork, unpinned HEAD --
 * tools/extras/install_warp_ctc.sh:8-11; cuDNN 5.1 -- tools/extras/
 * install_cudnn.sh) and no test in the reference pins their results (SURVEY
 * §4, §8c).  Against the reference itself parity is therefore UNPINNED.  This
 * restatement follows the published algorithms and the reference call sites,
 * and is cross-checked against torch fp64 (F.ctc_loss, nn.LSTM/GRU/RNN --
 * an independent implementation of the same published equations) through the
 * golden fixtures in tests/golden/ (generator: tests/golden/make_golden.py).
 *
 * Every function exists in a double (_f64) and a float (_f32) flavour.  The
 * _f64 flavour is the parity oracle; the _f32 flavour (OpenMP, blocked GEMM)
 * is the "port" CPU baseline timed by bench.py.
 */
#ifndef KALDI_CTC_ORACLE_H_
#define KALDI_CTC_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* RNN modes, numbering of CuDNNRecurrentComponent rnn-mode
 * (reference src/nnet2/nnet-cudnn-component.cc:252-259). */
enum { ORACLE_RNN_RELU = 0, ORACLE_RNN_TANH = 1, ORACLE_RNN_LSTM = 2, ORACLE_RNN_GRU = 3 };

/* ---------------- CTC (warp-ctc compute_ctc_loss semantics) ----------------
 * acts   [T_max][N][A] un-normalised activations (time-major, row t*N+n),
 *        exactly the affine output the reference hands to warp-ctc
 *        (src/ctc/ctc-nnet-update.cc:224-231).
 * grads  [T_max][N][A] (nullable) d(-log p)/d acts; rows t >= T_n are zero.
 * costs  [N] -log p(l_n | x_n); an infeasible utterance (L + repeats > T_n)
 *        gets cost 0 and zero gradient, as warp-ctc's CPU path returns. */
void oracle_ctc_f64(const double *acts, double *grads, const int *flat_labels,
                    const int *label_lengths, const int *input_lengths,
                    int A, int N, int T_max, double *costs, int blank);
void oracle_ctc_f32(const float *acts, float *grads, const int *flat_labels,
                    const int *label_lengths, const int *input_lengths,
                    int A, int N, int T_max, float *costs, int blank);

/* ---------------- cuDNN-v5 style recurrent layer ----------------
 * Parameter layout (reference nnet-cudnn-component.cc:270-413): for each
 * pseudo-layer p = layer*dirs + dir, the nlin matrices (ids 0..nlin/2-1 are
 * input weights W [H][Din], the rest recurrent R [H][H], row-major), then the
 * nlin bias vectors [H].  nlin = 8 (LSTM: i,f,c,o), 6 (GRU: r,z,h), 2 (RELU,
 * TANH).  Din = D for layer 0, dirs*H above. */
long oracle_rnn_params_size(int mode, int D, int H, int layers, int dirs);
long oracle_rnn_lin_offset(int mode, int D, int H, int layers, int dirs,
                           int pseudo_layer, int lin_id, int is_bias);
long oracle_rnn_reserve_size(int mode, int T, int N, int H, int layers, int dirs);

/* x [T][N][D], y [T][N][dirs*H] (fwd half in cols 0..H-1), hx = cx = 0.
 * All N sequences run the full T steps (no masking, as the reference's
 * cudnnRNNForwardTraining call, nnet-cudnn-component.cc:545-554). */
void oracle_rnn_forward_f64(int mode, int T, int N, int D, int H, int layers, int dirs,
                            const double *x, const double *w, double *y, double *reserve);
void oracle_rnn_forward_f32(int mode, int T, int N, int D, int H, int layers, int dirs,
                            const float *x, const float *w, float *y, float *reserve);
/* dy [T][N][dirs*H] -> dx [T][N][D] (nullable, overwritten) and dw (nullable,
 * ACCUMULATED, as cudnnRNNBackwardWeights). dhy = dcy = 0. */
void oracle_rnn_backward_f64(int mode, int T, int N, int D, int H, int layers, int dirs,
                             const double *x, const double *w, const double *y,
                             const double *dy, const double *reserve,
                             double *dx, double *dw);
void oracle_rnn_backward_f32(int mode, int T, int N, int D, int H, int layers, int dirs,
                             const float *x, const float *w, const float *y,
                             const float *dy, const float *reserve,
                             float *dx, float *dw);

/* ---------------- small ops ---------------- */
/* C[M][N] = alpha * op(A) op(B) + beta * C, row-major. */
void oracle_gemm_f64(int transA, int transB, int M, int N, int K, double alpha,
                     const double *A, int lda, const double *B, int ldb,
                     double beta, double *C, int ldc);
void oracle_gemm_f32(int transA, int transB, int M, int N, int K, float alpha,
                     const float *A, int lda, const float *B, int ldb,
                     float beta, float *C, int ldc);
/* Row argmax of the reference's CTC path: the GPU _find_row_max_id
 * (src/cudamatrix/cu-kernels.cu:2454-2500) -- 256-thread strided scan, then
 * a strict-greater shared-memory tree, so ties resolve by the tree (columns 1
 * and 2 equal -> 2); -1 when every value is <= -1e20 or NaN. */
void oracle_find_row_max_id_f32(const float *m, int rows, int cols, int *ids);
/* The CPU-only FindRowMaxId (src/cudamatrix/cu-matrix.cc:1630-1644): first
 * maximum above -1e21, else -1.  Not on the CTC path (kept for comparison). */
void oracle_find_row_max_id_cpu_f32(const float *m, int rows, int cols, int *ids);
/* SoftmaxComponent::Propagate (nnet-component.cc:929-946), floored at 1e-20 */
void oracle_softmax_rows_f32(const float *in, long rows, int cols, float *out);
/* CtcDecodableAmNnet (src/ctc/ctc-decodable-am-nnet.cc:28-80): blank skip,
 * floor, log, minus log prior (priors nullable), scale; returns rows kept */
int oracle_ctc_decodable_f32(const float *probs, int T, int A, const float *priors, float prob_scale,
                             float blank_threshold, float floor_v, float *out);
/* ComputeTotAccuracy (src/ctc/ctc-nnet-update.cc:261-317): returns sum_n L_n -
 * sum_n Levenshtein(ref_n, collapse(best ids)); *tot_weight = sum_n L_n. */
double oracle_ctc_accuracy(const int *best_ids, int T_max, int N,
                           const int *num_frames, const int *flat_labels,
                           const int *label_lengths, double *tot_weight);
int oracle_levenshtein(const int *a, int na, const int *b, int nb);

/* ---------------- whole nnet2 CTC train step ----------------
 * Topology of the recipe (egs/wsj/s5/steps/ctc/nnet2/components.py:73-102):
 * Splice(identity) -> [CuDNNRecurrent -> ClipGradient(norm)] x num_rnn ->
 * Affine(A).  One call = NnetCtcUpdater::ComputeForMinibatch with
 * nnet_to_update == nnet (src/ctc/ctc-nnet-update.cc:94-128): forward,
 * warp-ctc cost/grad, accuracy, backprop with the per-component in-place SGD
 * updates (dW of each RNN clipped to +-rnn_clip_gradient,
 * nnet-cudnn-component.cc:602-614; affine UpdateSimple,
 * nnet-component.cc:1190-1226).  ClipGradient self-repair is applied when
 * repair_draws[c] <= 0.5 and the cumulative clipped proportion exceeds
 * repair_threshold (nnet-cudnn-component.cc:980-1055); clip_num_clipped /
 * clip_count are the per-component cumulative counters (in/out). */
typedef struct {
  int num_rnn, mode, hidden, dirs, layers_per_rnn;
  int input_dim, num_targets;
  float clip_threshold;          /* ClipGradientComponent clipping-threshold */
  float repair_threshold;        /* self-repair-clipped-proportion-threshold */
  float repair_scale;            /* self-repair-scale (0 disables) */
  float repair_target;           /* self-repair-target */
  float rnn_clip_gradient;       /* CuDNNRecurrentComponent clip-gradient */
  float lr_rnn, lr_affine;
} oracle_nnet_spec;

/* rnn_params[c] points at component c's flat weights (updated in place);
 * affine_W [A][Dlast], affine_b [A] (updated in place).  feats [T][N][D].
 * Returns sum of costs; *tot_accuracy, *tot_weight as ComputeTotAccuracy. */
double oracle_train_step_f32(const oracle_nnet_spec *spec, float **rnn_params,
                             float *affine_W, float *affine_b, const float *feats,
                             int T, int N, const int *num_frames, const int *flat_labels,
                             const int *label_lengths, const float *repair_draws,
                             double *clip_num_clipped, double *clip_count,
                             double *tot_accuracy, double *tot_weight);
double oracle_train_step_f64(const oracle_nnet_spec *spec, double **rnn_params,
                             double *affine_W, double *affine_b, const double *feats,
                             int T, int N, const int *num_frames, const int *flat_labels,
                             const int *label_lengths, const float *repair_draws,
                             double *clip_num_clipped, double *clip_count,
                             double *tot_accuracy, double *tot_weight);

/* The same step, also returning the per-utterance costs [N], the network
 * output [T*N][A] and its best path [T*N] (each nullable). */
double oracle_train_step_ex_f32(const oracle_nnet_spec *spec, float **rnn_params,
                                float *affine_W, float *affine_b, const float *feats,
                                int T, int N, const int *num_frames, const int *flat_labels,
                                const int *label_lengths, const float *repair_draws,
                                double *clip_num_clipped, double *clip_count,
                                double *tot_accuracy, double *tot_weight,
                                double *costs_out, float *logits_out, int *ids_out);
double oracle_train_step_ex_f64(const oracle_nnet_spec *spec, double **rnn_params,
                                double *affine_W, double *affine_b, const double *feats,
                                int T, int N, const int *num_frames, const int *flat_labels,
                                const int *label_lengths, const float *repair_draws,
                                double *clip_num_clipped, double *clip_count,
                                double *tot_accuracy, double *tot_weight,
                                double *costs_out, double *logits_out, int *ids_out);

int oracle_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
