/*
 * kaldi_ctc_decode.h -- the decode-side use of a trained CTC model and the
 * validation objective, as a C ABI over gfx950 kernels
 * (csrc/decodable.hip) and the nnet2 trainer's forward pass.
 *
 *   kctc_softmax_rows        <- SoftmaxComponent::Propagate
 *                               (src/nnet2/nnet-component.cc:929-946; the
 *                               component steps/ctc/train.sh:471-477 appends
 *                               for decoding)
 *   kctc_ctc_decodable       <- CtcDecodableAmNnet's log-likelihood matrix
 *                               (src/ctc/ctc-decodable-am-nnet.cc:28-80)
 *   kctc_nnet_propagate      <- NnetComputation (src/nnet2/nnet-compute.cc),
 *                               N time-major sequences
 *   kctc_am_nnet_decodable   <- CtcDecodableAmNnet(trans_model, am_nnet, feats,
 *                               pad_input, prob_scale, blank_threshold)
 *   kctc_nnet_compute_prob   <- nnet2-ctc-compute-prob
 *                               (src/ctcbin/nnet2-ctc-compute-prob.cc:27-111)
 * Return 0 on success (kctc_last_error() describes a failure).
 */
#ifndef KALDI_CTC_AMD_KALDI_CTC_DECODE_H_
#define KALDI_CTC_AMD_KALDI_CTC_DECODE_H_

#include <stddef.h>

#include "kaldi_ctc_train.h"

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;

/* out[r] = softmax(in[r]) (max-subtracted), floored at 1e-20; device, row-major */
int kctc_softmax_rows(struct ihipStream_t *stream, const float *in, long rows, int cols, float *out);

/* probs [T][A] (device; the output of a model ending in SoftmaxComponent) ->
 * out [*num_kept][A] (device):
 *   blank_threshold < 1: only frames t with probs[t][0] < blank_threshold, in
 *     order (all frames if none qualifies, as the reference warns and does);
 *   v = log(max(p, floor_value))   (1e-10 CtcDecodableAmNnet, 1e-20 ...Parallel)
 *   v -= log(priors[a])            (priors: linear, device, nullable)
 *   v *= prob_scale
 * scratch: kctc_ctc_decodable_scratch_bytes(T) bytes of device memory.
 * Synchronises the stream to return *num_kept. */
size_t kctc_ctc_decodable_scratch_bytes(int T);
int kctc_ctc_decodable(struct ihipStream_t *stream, const float *probs, int T, int A, const float *priors,
                       float prob_scale, float blank_threshold, float floor_value, float *out, void *scratch,
                       int *num_kept);

/* forward pass of the whole network: feats_dev [T_max*N*num_splice][input_dim]
 * (FormatNnetInput layout, num_splice = 1 + left + right context,
 * kctc_nnet_context; the caller's buffer must hold that many rows) ->
 * out_dev [T_max*N][output_dim] (device), len = T_max*N*output_dim */
int kctc_nnet_propagate(kctcNnet_t nnet, const float *feats_dev, int T_max, int N, float *out_dev, long len);

/* CtcDecodableAmNnet for one utterance feats_dev [T][input_dim] (plain
 * feature rows) with the model's priors (an nnet2-ctc model file read by
 * kctc_am_nnet_read), pad_input = true (the reference's default): a network
 * with frame context sees the first / last frame repeated LeftContext /
 * RightContext times (NnetComputer, src/nnet2/nnet-compute.cc:64-90), so T
 * frames give T rows.  Writes the kept rows of the [T][A] log-likelihood
 * matrix to out_host (capacity T*A floats), *num_rows = rows kept. */
int kctc_am_nnet_decodable(kctcNnet_t nnet, const float *feats_dev, int T, float prob_scale,
                           float blank_threshold, float *out_host, int *num_rows);

/* nnet2-ctc-compute-prob over an egs archive (binary "ark:"): examples in
 * batches of 10 in archive order, every example used (no training skip
 * rules), ComputeNnetObjf per batch (forward + CTC + best-path accuracy, no
 * update).  Outputs: examples, total objective (sum of -log p; the CLI prints
 * tot_like / tot_weight), total accuracy, total weight (sum of labels). */
int kctc_nnet_compute_prob(kctcNnet_t nnet, const char *rspecifier, long *num_examples, double *tot_like,
                           double *tot_accuracy, double *tot_weight);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_KALDI_CTC_DECODE_H_ */
