// clipgrad.h -- ClipGradientComponent backprop + self-repair on device.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace kctc {

struct ClipState {  // device-resident; cumulative like the component's members
  int step_clipped;
  int pad;
  double num_clipped, count, num_self_repaired;
  double dn, rn, scale, dn2;
  int active;
  int pad2;
};

size_t clipgrad_scratch_bytes(long rows);
// d [rows][dim] in place.  try_repair = the host-side part of RepairGradients'
// gate (threshold < 1, scale != 0, count_ != 0, RandUniform() <= 0.5); the
// clipped-proportion part is evaluated on the device.
void clipgrad_backprop(hipStream_t s, float *d, const float *in_value, long rows, int dim,
                       float threshold, bool norm_based, bool try_repair, float repair_threshold,
                       float repair_target, float repair_scale, ClipState *st, void *scratch,
                       const ClipState *decide = nullptr);
// st accumulates the counters; decide (default st) supplies the clipped
// proportion of the repair decision: the backpropped component's own stats,
// which differ from to_update's under momentum (ctc-nnet-train.cc:194-202).

}  // namespace kctc
