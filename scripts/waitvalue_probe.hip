// waitvalue_probe.hip -- does hipStreamWaitValue32 release a stream when a
// kernel on another stream stores the value (a) into hipMallocSignalMemory,
// (b) into plain hipMalloc memory?  Prints the order of the two kernels'
// completion stamps.  Build: hipcc --offload-arch=gfx950 -O2 waitvalue_probe.hip -o waitvalue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("%s -> %s\n", #x, hipGetErrorString(e));                           \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void late_store(unsigned *word, unsigned v, unsigned long long *stamp, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
  stamp[0] = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void mark(unsigned long long *stamp) { stamp[1] = __builtin_amdgcn_s_memrealtime(); }

static int run(const char *name, unsigned *word) {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  unsigned long long *st;
  CK(hipMalloc(&st, 64));
  CK(hipMemset(st, 0, 64));
  CK(hipMemset(word, 0, 4));
  CK(hipDeviceSynchronize());
  hipError_t e = hipStreamWaitValue32(a, word, 5u, hipStreamWaitValueGte, 0xFFFFFFFFu);
  if (e != hipSuccess) {
    printf("%s: hipStreamWaitValue32 -> %s\n", name, hipGetErrorString(e));
    return 0;
  }
  hipLaunchKernelGGL(mark, dim3(1), dim3(1), 0, a, st);
  hipLaunchKernelGGL(late_store, dim3(1), dim3(1), 0, b, word, 5u, st, 2000000ull);  // 20 ms
  CK(hipDeviceSynchronize());
  unsigned long long h[2];
  CK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
  printf("%s: store at %llu, waiter ran at %llu: %s (gap %.1f us)\n", name, h[0], h[1],
         h[1] >= h[0] ? "released after the store" : "NOT GATED", ((double)h[1] - (double)h[0]) * 0.01);
  (void)hipFree(st);
  return 0;
}

int main() {
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
  unsigned *sig = nullptr, *dev = nullptr;
  CK(hipExtMallocWithFlags((void **)&sig, 64, hipMallocSignalMemory));
  CK(hipMalloc(&dev, 64));
  if (run("signal memory", sig)) return 1;
  if (run("device memory", dev)) return 1;
  return 0;
}
