/*
 * kaldi_ctc_train.h -- C ABI of the native nnet2 CTC trainer (csrc/nnet.cpp).
 *
 * The C++ side mirrors the reference's nnet2 classes on device buffers
 * (kctc::nnet2::{Component, SpliceComponent, CuDNNRecurrentComponent,
 * ClipGradientComponent, AffineComponent, Nnet, NnetCtcUpdater}); this ABI is
 * what a ctypes/cgo/JNI host binds.  Each entry names the reference function it
 * replaces:
 *   kctc_nnet_create        <- nnet-init / Nnet::Init from component config lines
 *                              (src/nnet2/nnet-nnet.cc; line format of
 *                              egs/wsj/s5/steps/ctc/nnet2/components.py:73-102)
 *   kctc_nnet_train_step    <- DoBackprop(nnet, egs, &formatted, nnet, &acc)
 *                              == NnetCtcUpdater::ComputeForMinibatch + SGD
 *                              (src/ctc/ctc-nnet-update.cc:94-128, 447-463)
 *   kctc_nnet_compute_objf  <- ComputeNnetObjf (no backprop; nnet2-ctc-compute-prob,
 *                              src/ctc/ctc-nnet-update.cc:426-431)
 *   kctc_nnet_get/set_params<- UpdatableComponent::Vectorize / UnVectorize
 *   kctc_nnet_write/read    <- Nnet::Write / Read (nnet-nnet.cc:170-220; component tokens of
 *                              nnet-cudnn-component.cc:673-837, nnet-component.cc:1228-1274,
 *                              2797-2831), Kaldi text or binary mode
 *   kctc_am_nnet_*          <- CtcTransitionModel + AmNnet model files (am-nnet.cc:31-55)
 *   kctc_format_input       <- FormatNnetInput (src/ctc/ctc-nnet-update.cc:351-424)
 *   kctc_nnet_enable_dp     <- (new) data parallelism: RCCL all-reduce of the
 *                              weight gradients over xGMI; replaces the recipe's
 *                              per-iteration model averaging (nnet-am-average)
 * Features are device pointers in the time-major [T_max*N*num_splice][dim]
 * layout of FormatNnetInput (num_splice = 1 for context-free networks);
 * labels/lengths are host arrays.  Return 0 on success,
 * non-zero on error (kctc_last_error() describes it).
 */
#ifndef KALDI_CTC_AMD_KALDI_CTC_TRAIN_H_
#define KALDI_CTC_AMD_KALDI_CTC_TRAIN_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;
typedef struct kctcNnetImpl *kctcNnet_t;

const char *kctc_last_error(void);

/* config: newline-separated component lines ("<Type> key=value ...").
 * seed: weight-init RNG seed.  device: HIP device ordinal. */
int kctc_nnet_create(kctcNnet_t *nnet, const char *config, unsigned long long seed, int device);
int kctc_nnet_destroy(kctcNnet_t nnet);
int kctc_nnet_num_components(kctcNnet_t nnet);
/* Nnet::LeftContext / RightContext (src/nnet2/nnet-nnet.cc:52-73).  The
 * network input of a minibatch is FormatNnetInput's layout for num_splice =
 * 1 + left + right: [T_max*N*num_splice][input_dim], row (t*N+n)*num_splice+s
 * = frame t+s of utterance n (src/ctc/ctc-nnet-update.cc:351-424); the
 * train/objf calls take T_max = output frames and num_frames = the CTC input
 * lengths (NumFrames - left_context - right context, :187-195). */
int kctc_nnet_context(kctcNnet_t nnet, int *left, int *right);
/* writes "<Type> dim info" of component c into buf */
int kctc_nnet_component_info(kctcNnet_t nnet, int c, char *buf, size_t buflen);
long kctc_nnet_num_params(kctcNnet_t nnet, int c);
int kctc_nnet_get_params(kctcNnet_t nnet, int c, float *host, long n);
int kctc_nnet_set_params(kctcNnet_t nnet, int c, const float *host, long n);
/* the gradient component c's last update used, before its clip (the
 * summed one under data parallelism), in Vectorize order */
int kctc_nnet_get_grad(kctcNnet_t nnet, int c, float *host, long n);
int kctc_nnet_set_learning_rate(kctcNnet_t nnet, float lr);
/* ClipGradientComponent counters of component c: num_clipped, count */
int kctc_nnet_clip_stats(kctcNnet_t nnet, int c, double *num_clipped, double *count);
/* srand(seed) of the trainer's rand() stream (nnet2-ctc-train-simple --srand,
 * src/ctcbin/nnet2-ctc-train-simple.cc:47,69; 0 when never called).  The only
 * consumer on this path is ClipGradientComponent self-repair: one RandUniform()
 * = (rand() + 1.0) / (RAND_MAX + 2.0) per ClipGradient Backprop, top component
 * first, drawn only when the reference's short-circuit conditions reach it
 * (src/nnet2/nnet-cudnn-component.cc:987-991) -- the same glibc generator, so
 * the repair decisions equal the reference's for the same --srand.
 * kctc_nnet_rand_calls: rand() calls made so far. */
int kctc_nnet_srand(kctcNnet_t nnet, unsigned seed);
int kctc_nnet_rand_calls(kctcNnet_t nnet, long *calls);
/* The last finished minibatch's best path (FindRowMaxId of the network
 * output, [T_max*N] int32, row t*N+n; the ids ComputeTotAccuracy collapsed)
 * and its network output ([T_max*N][A] fp32; valid until the next step is
 * queued).  len must equal T_max*N (ids) / T_max*N*A (output). */
int kctc_nnet_last_best_path(kctcNnet_t nnet, int *ids, long len);
/* per-utterance costs (-log p(l_n | x_n), warp-ctc `costs`) of that minibatch */
int kctc_nnet_last_costs(kctcNnet_t nnet, double *costs, int N);
int kctc_nnet_last_output(kctcNnet_t nnet, float *host, long len);

/* One SGD minibatch.  feats_dev [T_max*N*num_splice][input_dim] (device,
 * zero padded; num_splice = 1 + left + right context of kctc_nnet_context,
 * 1 for the recipe's networks): the call reads exactly that many rows, so a
 * buffer laid out for another context is an out-of-bounds read, not an error
 * the library can see.  Outputs: sum of CTC costs, accuracy numerator
 * (sum L - edits), weight (sum L). */
int kctc_nnet_train_step(kctcNnet_t nnet, const float *feats_dev, int T_max, int N,
                         const int *num_frames, const int *flat_labels, const int *label_lengths,
                         double *tot_objf, double *tot_accuracy, double *tot_weight);
/* kctc_nnet_train_step split in two for a pipelined host loop: queues the
 * minibatch's device work (feats_dev must stay valid until its stats come
 * back) and, once two are queued, waits for the older one and returns ITS
 * stats with *have_stats = 1 (else *have_stats = 0).  kctc_nnet_train_flush
 * returns the remaining ones, one per call, until *have_stats = 0.  The
 * updates are the same as kctc_nnet_train_step's; only the host waits move
 * (TrainNnetSimple's per-minibatch stats are reported one minibatch late). */
int kctc_nnet_train_step_async(kctcNnet_t nnet, const float *feats_dev, int T_max, int N,
                               const int *num_frames, const int *flat_labels, const int *label_lengths,
                               int *have_stats, double *tot_objf, double *tot_accuracy, double *tot_weight);
int kctc_nnet_train_flush(kctcNnet_t nnet, int *have_stats, double *tot_objf, double *tot_accuracy,
                          double *tot_weight);

/* ComputeNnetObjf: the same input layout as kctc_nnet_train_step, no update */
int kctc_nnet_compute_objf(kctcNnet_t nnet, const float *feats_dev, int T_max, int N,
                           const int *num_frames, const int *flat_labels,
                           const int *label_lengths, double *tot_objf, double *tot_accuracy,
                           double *tot_weight);
/* The stream the trainer's kernels run on (for host-side event timing). */
struct ihipStream_t *kctc_nnet_stream(kctcNnet_t nnet);
/* Per-launch device time of the last step's kernels, by kernel family (ms):
 * filled only when profiling is enabled with kctc_nnet_set_profiling(nnet, 1). */
int kctc_nnet_set_profiling(kctcNnet_t nnet, int on);
int kctc_nnet_profile(kctcNnet_t nnet, const char *family, double *ms_total, int *launches);

int kctc_nnet_write(kctcNnet_t nnet, const char *path);  /* text mode */
/* Nnet::Write in Kaldi text (binary = 0) or binary ("\0B" header) mode */
int kctc_nnet_write_kaldi(kctcNnet_t nnet, const char *path, int binary);
/* either mode (detected from the "\0B" header) */
int kctc_nnet_read(kctcNnet_t *nnet, const char *path, int device);

/* nnet2-ctc model files, the <model-in> / <model-out> of nnet2-ctc-train-simple
 * (src/ctcbin/nnet2-ctc-train-simple.cc:58-77): CtcTransitionModel
 * (src/ctc/ctc-transition-model.h:83-90, kept as the opaque bytes it was read
 * as and written back unchanged) then AmNnet::Write = Nnet + priors
 * (src/nnet2/am-nnet.cc:31-42).  Read detects the mode; a model whose
 * transition model was read in one mode must be written in that mode. */
int kctc_am_nnet_read(kctcNnet_t *nnet, const char *path, int device);
int kctc_am_nnet_write(kctcNnet_t nnet, const char *path, int binary);
int kctc_am_nnet_num_priors(kctcNnet_t nnet);
int kctc_am_nnet_get_priors(kctcNnet_t nnet, float *priors, int dim);
/* AmNnet::SetPriors (am-nnet.cc:44-55): dim <= output dim, zero-extended */
int kctc_am_nnet_set_priors(kctcNnet_t nnet, const float *priors, int dim);

/* Data parallelism over RCCL (one process per GPU).  uid: 128-byte
 * ncclUniqueId from kctc_dp_unique_id on rank 0, broadcast by the launcher. */
int kctc_dp_unique_id(void *uid128);
/* world_size >= 1 (a one-rank communicator is valid and runs the same
 * all-reduce path); world_size 0 switches data parallelism off. */
int kctc_nnet_enable_dp(kctcNnet_t nnet, const void *uid128, int rank, int world_size);
/* The same exchange over a host transport: each component's gradient bucket
 * is copied to pinned host memory on the comm stream, `allreduce(buf, n,
 * user)` sums it in place across the ranks (e.g. gloo), and it is copied back;
 * the updates then run exactly as with RCCL.  For hosts without RCCL peers
 * (several processes sharing one GPU, CPU-side rendezvous). */
typedef void (*kctc_host_allreduce_fn)(float *buf, long n, void *user);
int kctc_nnet_enable_dp_host(kctcNnet_t nnet, kctc_host_allreduce_fn allreduce, void *user, int world_size);
/* Data-parallel mode.  0 (default): the gradient of every step is summed over
 * the ranks before the update (kctc_nnet_enable_dp).  1: model averaging --
 * the ranks step independently and kctc_nnet_average_params replaces every
 * updatable component's parameters by their mean over the ranks: the recipe's
 * per-iteration nnet-am-average (egs/wsj/s5/steps/ctc/train.sh:434-435,
 * src/nnet2bin/nnet-am-average.cc:185-241, default weights 1/num-models),
 * e.g. called every K minibatches.  ClipGradient counters and momentum
 * deltas stay per rank (nnet-am-average only averages updatable components). */
int kctc_nnet_set_dp_mode(kctcNnet_t nnet, int mode);
int kctc_nnet_average_params(kctcNnet_t nnet);

/* A step whose device error word is set on ANY rank (a recurrence's bounded
 * spin timed out) is skipped on every rank: the word is summed over the ranks
 * through the exchange after the gradient buckets, before the updates, and
 * the train step then fails on every rank with the parameters unchanged.
 * Test hook: the next minibatch of `nnet` starts with error word `word`. */
int kctc_nnet_inject_step_error(kctcNnet_t nnet, unsigned word);

/* CU budget.  RCCL's kernels are capped at KCTC_COMM_CTAS
 * blocks (default 16, ncclConfig_t.maxCTAs) and the streamed GEMMs beside a
 * backward recurrence leave that many CUs free.  kctc_nnet_enable_cu_probe is
 * the test of that budget: a one-rank exchange whose every gradient bucket
 * launches a kernel holding `blocks` whole CUs for `usec` microseconds on the
 * comm stream (gradients untouched); blocks 0 switches it off. */
int kctc_nnet_enable_cu_probe(kctcNnet_t nnet, int blocks, double usec);
/* Ranks sharing one device (host-transport data parallelism on one GPU):
 * the nnets created afterwards in this process run on CU-masked streams
 * holding CU share `part` of `nparts`, and the persistent kernels size
 * themselves for that share.  Call before kctc_nnet_create. */
int kctc_set_cu_partition(int part, int nparts);
/* Check of the shares: runs 8 blocks per CU on a stream masked to share
 * `part` of `nparts` (the mask kctc_set_cu_partition builds) and returns the
 * distinct CUs they ran on as (XCC_ID << 16) | HW_ID[15:8] (CU, SH, SE) in
 * ids[0 .. *n_ids) (at most max_ids).  Test support; synchronous. */
int kctc_cu_partition_probe(int part, int nparts, unsigned *ids, int max_ids, int *n_ids);

/* Arithmetic of every CuDNNRecurrentComponent's recurrences and gate GEMMs:
 * 0 fp32-class (default), 1 bf16 operands with fp32 accumulation and fp32
 * master weights (BASELINE configs[4]).  Affine, CTC and the updates stay
 * fp32; model files are unaffected. */
int kctc_nnet_set_precision(kctcNnet_t nnet, int precision);

/* TrainNnetSimple momentum (src/ctc/ctc-nnet-train.cc:194-245, config
 * ctc-nnet-train.h:33-66): with m != 0 every update goes to a delta copy
 * (delta += lr * clip(grad); params += delta; delta *= m) and ClipGradient
 * counters accumulate in the delta copy.  0 (default) = plain SGD. */
int kctc_nnet_set_momentum(kctcNnet_t nnet, float momentum);

/* TrainNnetSimple (src/ctc/ctc-nnet-train.cc:185-284) over a background egs
 * reader (include/kaldi_ctc_egs.h, opened with the trainer's minibatch_size /
 * max_allow_frames): every minibatch is formatted on the GPU and trained with
 * DoBackprop until the archive is exhausted or max_minibatches (> 0) have run.
 * Outputs (may be NULL): examples processed, total weight (labels), total
 * objective, total accuracy. */
struct kctcEgsReader_;
int kctc_nnet_train_simple(kctcNnet_t nnet, struct kctcEgsReader_ *reader, long max_minibatches,
                           long *num_egs, double *tot_weight, double *tot_objf, double *tot_accuracy);

/* LevenshteinEditDistance with unit costs (src/util/edit-distance-inl.h), as
 * ComputeTotAccuracy uses it (src/ctc/ctc-nnet-update.cc:261-317), by Myers'
 * bit-vector algorithm (ref in ceil(nref/64) 64-bit words; O(nhyp*nref/64)). */
int kctc_levenshtein(const int *ref, int nref, const int *hyp, int nhyp);

/* FormatNnetInput: pack per-utterance [T_n][dim] host matrices (concatenated
 * in `feats`, row offsets by num_frames) into [T_max*N][dim], row t*N+n,
 * zero padded.  out must hold T_max*N*dim floats (host). */
int kctc_format_input(const float *feats, const int *num_frames, int N, int dim, int T_max,
                      float *out);

/* Synthetic minibatch of the BASELINE.md §2 generator (splitmix64 + Box-Muller,
 * seed = 20161015 + 1000*rank + step): features N(0,1) already formatted
 * [T_max*N][dim] (host), T_n = T_max - floor(u*0.1*T_max) (n=0 gets T_max),
 * L_n = floor(T_n*label_ratio) clamped to <= 639 and <= (T_n-1)/2, labels
 * uniform in [1, A-1] without consecutive repeats.  flat_labels capacity
 * >= N*639.  Returns the total number of labels. */
long kctc_synth_minibatch(unsigned long long seed, int T_max, int N, int dim, int A,
                          double label_ratio, float *feats, int *num_frames, int *flat_labels,
                          int *label_lengths);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_KALDI_CTC_TRAIN_H_ */
