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
// DPP reductions (VALU lane permutes, no LDS round trip as __shfl_xor's
// ds_bpermute): max over each aligned group of 8 / 16 lanes, result in every
// lane of the group; and the full-wave max, result in lane 63.
#define KCTC_DPP(v, ctrl, rm) \
  __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), ctrl, rm, 0xF, false))
__device__ __forceinline__ float group_max8(float v) {
  v = fmaxf(v, KCTC_DPP(v, 0xB1, 0xF));   // quad_perm(1,0,3,2)
  v = fmaxf(v, KCTC_DPP(v, 0x4E, 0xF));   // quad_perm(2,3,0,1)
  v = fmaxf(v, KCTC_DPP(v, 0x141, 0xF));  // row_half_mirror
  return v;
}
__device__ __forceinline__ float group_max16(float v) {
  v = group_max8(v);
  return fmaxf(v, KCTC_DPP(v, 0x140, 0xF));  // row_mirror
}
__device__ __forceinline__ float wave_max_l63(float v) {
  v = group_max16(v);
  v = fmaxf(v, KCTC_DPP(v, 0x142, 0xA));  // row_bcast15 into rows 1, 3
  v = fmaxf(v, KCTC_DPP(v, 0x143, 0xC));  // row_bcast31 into rows 2, 3
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
