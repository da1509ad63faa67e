// prof.h -- optional per-kernel timing with hipEvents on the launch stream
// (implemented by CuDevice in nnet.cpp; no-ops unless profiling is enabled).
#pragma once
#include <hip/hip_runtime.h>

namespace kctc {
void prof_begin(hipStream_t s, const char *family);
void prof_end(hipStream_t s);
struct ProfSpan {
  hipStream_t s;
  ProfSpan(hipStream_t st, const char *f) : s(st) { prof_begin(s, f); }
  ~ProfSpan() { prof_end(s); }
};
}  // namespace kctc
