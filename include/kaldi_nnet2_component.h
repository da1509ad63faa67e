/*
 * kaldi_nnet2_component.h -- C ABI of the nnet2 Component plug-in point
 * (src/nnet2/nnet-component.h:157-348) for the components of the CTC path:
 * SpliceComponent, CuDNNRecurrentComponent (HIP recurrences, csrc/rnn.hip),
 * ClipGradientComponent, AffineComponent and SoftmaxComponent.
 *
 * Each entry names the reference member it replaces:
 *   kctc_component_init        <- Component::NewComponentOfType + InitFromString
 *                                 (nnet-component.cc:52-120; config line
 *                                 "<Type> key=value ...", the nnet-init form)
 *   kctc_component_read/write  <- Component::ReadNew / Write (nnet-component.cc:38-48)
 *   kctc_component_copy        <- Component::Copy
 *   kctc_component_propagate   <- Component::Propagate(in_info, out_info, in, out)
 *   kctc_component_backprop    <- Component::Backprop(in_info, out_info, in_value,
 *                                 out_value, out_deriv, to_update, in_deriv)
 *   kctc_component_set_zero    <- UpdatableComponent::SetZero(treat_as_gradient)
 *   kctc_component_dot_product <- UpdatableComponent::DotProduct
 *   kctc_component_perturb_params <- UpdatableComponent::PerturbParams
 *   kctc_component_scale/add   <- UpdatableComponent::Scale / Add
 *                                 (ClipGradientComponent / SoftmaxComponent:
 *                                 their statistics' Scale / Add)
 *   kctc_component_get/set_params <- Vectorize / UnVectorize
 *   kctc_nnet_get/set_component <- Nnet::GetComponent(c).Copy() / Nnet::SetComponent
 *                                 (nnet-nnet.cc:659-665)
 *   kctc_nnet_scale_params / kctc_nnet_add_params / kctc_nnet_average_models
 *                               <- the per-component loops of nnet-am-average
 *                                 (src/nnet2bin/nnet-am-average.cc:185-241)
 *
 * Layout: matrices are device pointers, row-major with NumCols() == Stride(),
 * time-major rows t*N + n (N sequences of T frames, the FormatNnetInput
 * layout).  A component whose Context() spans num_splice = last - first + 1
 * frames (SpliceComponent) reads num_splice input rows per output frame:
 * input rows (t*N+n)*num_splice + s.  Lengths are element counts and are
 * checked.  Every call is synchronous: it runs on the handle's own HIP stream
 * and waits for it before returning, so buffers written on another stream must
 * be complete before the call.  Return 0 on success, non-zero on error
 * (kctc_last_error() describes it).
 *
 * Backprop follows the reference's semantics exactly: when to_update is
 * non-NULL its parameters are updated immediately inside the call
 * (CuDNNRecurrentComponent: dW clipped to +-clip-gradient, then W += lr * dW,
 * nnet-cudnn-component.cc:558-614; AffineComponent::UpdateSimple,
 * nnet-component.cc:1184-1226), so after SetZero(treat_as_gradient = 1) it
 * holds the gradient.  As with cuDNN's reserve space, a CuDNNRecurrentComponent
 * must have run Propagate on the same input (same T, N) before its Backprop.
 */
#ifndef KALDI_CTC_AMD_KALDI_NNET2_COMPONENT_H_
#define KALDI_CTC_AMD_KALDI_NNET2_COMPONENT_H_

#include <stddef.h>

#include "kaldi_ctc_train.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kctcComponentImpl *kctcComponent_t;

int kctc_component_init(kctcComponent_t *c, const char *config_line, unsigned long long seed, int device);
int kctc_component_read(kctcComponent_t *c, const char *path, int device);
int kctc_component_write(kctcComponent_t c, const char *path, int binary);
int kctc_component_copy(kctcComponent_t c, kctcComponent_t *copy);
int kctc_component_destroy(kctcComponent_t c);

/* "SpliceComponent", ... */
int kctc_component_type(kctcComponent_t c, char *buf, size_t buflen);
int kctc_component_info(kctcComponent_t c, char *buf, size_t buflen);
int kctc_component_dims(kctcComponent_t c, int *input_dim, int *output_dim);
/* Context() offsets (at most cap); *n = their number */
int kctc_component_context(kctcComponent_t c, int *offsets, int cap, int *n);
int kctc_component_backprop_needs(kctcComponent_t c, int *needs_input, int *needs_output);
int kctc_component_is_updatable(kctcComponent_t c);

/* in: [T*N*num_splice][InputDim], out: [T*N][OutputDim] */
int kctc_component_propagate(kctcComponent_t c, int T, int N, const float *in, long in_len, float *out,
                             long out_len);
/* in_value / out_value may be NULL when BackpropNeeds{Input,Output} say so;
 * to_update and in_deriv may be NULL; in_deriv may alias out_deriv for
 * components of equal input and output dimension. */
int kctc_component_backprop(kctcComponent_t c, int T, int N, const float *in_value, long in_len,
                            const float *out_value, long out_len, const float *out_deriv, long out_deriv_len,
                            kctcComponent_t to_update, float *in_deriv, long in_deriv_len);

/* UpdatableComponent */
long kctc_component_num_params(kctcComponent_t c);
int kctc_component_get_params(kctcComponent_t c, float *host, long n);
int kctc_component_set_params(kctcComponent_t c, const float *host, long n);
int kctc_component_learning_rate(kctcComponent_t c, float *lr);
int kctc_component_set_learning_rate(kctcComponent_t c, float lr);
int kctc_component_is_gradient(kctcComponent_t c);
int kctc_component_set_zero(kctcComponent_t c, int treat_as_gradient);
/* fp64 accumulation on the device */
int kctc_component_dot_product(kctcComponent_t c, kctcComponent_t other, double *dot);
int kctc_component_perturb_params(kctcComponent_t c, float stddev);
int kctc_component_scale(kctcComponent_t c, float scale);
int kctc_component_add(kctcComponent_t c, float alpha, kctcComponent_t other);
/* seed of the PerturbParams noise stream (each call draws fresh noise) */
int kctc_set_perturb_seed(unsigned long long seed);
/* ClipGradientComponent: srand() of the handle's own rand() stream that
 * self-repair draws from (a handle starts with srand(0)) */
int kctc_component_srand(kctcComponent_t c, unsigned seed);

/* Components of a network: a copy of component `index` on the network's
 * device, and the replacement of component `index` by a copy of `c`. */
int kctc_nnet_get_component(kctcNnet_t nnet, int index, kctcComponent_t *c);
int kctc_nnet_set_component(kctcNnet_t nnet, int index, kctcComponent_t c);

/* nnet-am-average's loops over components [0, c_end) (c_end = the last
 * updatable component when skip_last_layer, else all): UpdatableComponent
 * Scale / Add and the SoftmaxComponent statistics' Scale / Add.
 * kctc_nnet_average_models: nnets[0] = sum_i weights[i] * nnets[i] (weights
 * NULL: 1/num each), nnets[0] scaled first, then the others added in order. */
int kctc_nnet_scale_params(kctcNnet_t nnet, float scale, int skip_last_layer);
int kctc_nnet_add_params(kctcNnet_t nnet, float alpha, kctcNnet_t other, int skip_last_layer);
int kctc_nnet_average_models(kctcNnet_t *nnets, const float *weights, int num, int skip_last_layer);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_KALDI_NNET2_COMPONENT_H_ */
