// decodable.h -- decode-side kernels (decodable.hip): SoftmaxComponent
// forward and the CtcDecodableAmNnet log-likelihood matrix.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace kctc {

// out = softmax of each row of in (max-subtracted), floored at 1e-20
void softmax_rows(hipStream_t s, const float *in, long rows, int cols, float *out);
// SoftmaxComponent::Backprop: out = value * (deriv - rowdot(value, deriv))
void diff_softmax_rows(hipStream_t s, const float *value, const float *deriv, long rows, int cols, float *out);
// probs [T][A] -> out [kept][A] (see decodable.hip); priors: linear, device,
// nullable; scratch >= ctc_decodable_scratch_bytes(T); *kept_dev (device int)
size_t ctc_decodable_scratch_bytes(int T);
void ctc_decodable(hipStream_t s, const float *probs, int T, int A, const float *priors, float prob_scale,
                   float blank_threshold, float floor_v, float *out, void *scratch, int *kept_dev);

}  // namespace kctc
