// test_hooks.cpp -- C ABI of csrc/test_hooks.h (measurement / test entry
// points outside the drop-in headers).
#include "test_hooks.h"

#include <stdexcept>

#include "common.h"
#include "gemm.h"

extern "C" {

float kcm_bench_gemm_packed(struct ihipStream_t *stream, int M, int N, int K, int bf16, int iters, int split) {
  if (M <= 0 || N <= 0 || K <= 0 || iters <= 0) return -1.f;
  try {
    return kctc::x3p_bench(stream, M, N, K, bf16 != 0, iters, split);
  } catch (...) {
    return -1.f;
  }
}

int kcm_test_row_stream(struct ihipStream_t *stream, int M, int N, int K, int forward, int tail_rows,
                        const float *E, const float *Wt, const float *bias, float *C) {
  if (!E || !Wt || !C || M <= 0 || N <= 0 || K <= 0 || K % 32) return 1;
  try {
    kctc::x3p_row_stream_selftest(stream, M, N, K / 32, forward, tail_rows, E, Wt, bias, C);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  } catch (const std::invalid_argument &) {
    return 1;
  } catch (...) {
    return 3;
  }
}

}  // extern "C"
