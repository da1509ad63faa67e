// common.h -- shared helpers for the kaldi-ctc MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace kctc {

constexpr int kWave = 64;  // CDNA wavefront

struct HipError : std::runtime_error {
  explicit HipError(const std::string &s) : std::runtime_error(s) {}
};

#define KCTC_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      throw ::kctc::HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " @" \
                             + __FILE__ + ":" + std::to_string(__LINE__));            \
  } while (0)

#define KCTC_REQUIRE(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) throw std::invalid_argument(std::string(msg));   \
  } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

}  // namespace kctc
