// cumask_probe.hip -- which XCD / CU a hipExtStreamCreateWithCUMask bit
// selects on this device (for the comm stream's mask, rnn.h
// rnn_set_comm_masked).  For each probed mask bit b, 16 blocks run on a
// stream masked to {b} and write their XCC_ID and HW_ID; the program prints
// "bit b -> xcc x cu c" lines, then the XCDs a mask of bits {b : b % 8 >= 4}
// reaches.  Build: hipcc --offload-arch=gfx950 -O2 cumask_probe.hip -o cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void where_kernel(unsigned *out) {
  if (threadIdx.x) return;
  unsigned x, h;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
  out[2 * blockIdx.x] = x;
  out[2 * blockIdx.x + 1] = h;
}

static int run(const std::vector<unsigned> &mask, int blocks, unsigned *dev, std::vector<unsigned> &host) {
  hipStream_t s;
  CK(hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()));
  hipLaunchKernelGGL(where_kernel, dim3(blocks), dim3(64), 0, s, dev);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(host.data(), dev, sizeof(unsigned) * 2 * blocks, hipMemcpyDeviceToHost));
  CK(hipStreamDestroy(s));
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("cus %d\n", cus);
  const int words = (cus + 31) / 32, blocks = 16;
  unsigned *dev;
  CK(hipMalloc(&dev, sizeof(unsigned) * 2 * 1024));
  std::vector<unsigned> host(2 * 1024);
  const int bits[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 31, 32, 33, 63, 64, 127, 128, 200, 255};
  for (int b : bits) {
    if (b >= cus) continue;
    std::vector<unsigned> m(words, 0u);
    m[b / 32] = 1u << (b % 32);
    if (run(m, blocks, dev, host)) return 1;
    // HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] ...
    unsigned xs = 0;
    for (int i = 0; i < blocks; i++) xs |= 1u << (host[2 * i] & 15);
    const unsigned h = host[1];
    printf("bit %3d -> xcc mask 0x%02x  cu %u sh %u se %u\n", b, xs, (h >> 8) & 15, (h >> 12) & 1, (h >> 13) & 7);
  }
  for (int variant = 0; variant < 2; variant++) {
    std::vector<unsigned> m(words, 0u);
    for (int b = 0; b < cus; b++) {
      const bool on = variant == 0 ? (b % 8) >= 4 : b >= cus / 2;
      if (on) m[b / 32] |= 1u << (b % 32);
    }
    if (run(m, 1024, dev, host)) return 1;
    unsigned cnt[16] = {0};
    for (int i = 0; i < 1024; i++) cnt[host[2 * i] & 15]++;
    printf("%s:", variant == 0 ? "mask b%8>=4" : "mask b>=cus/2");
    for (int x = 0; x < 8; x++) printf(" %u", cnt[x]);
    printf("\n");
  }
  // block b -> XCC of b % 8 over repeated launches (odd grids in between)
  for (int rep = 0; rep < 4; rep++) {
    std::vector<unsigned> m(words, 0xffffffffu);
    if (run(m, 3 + rep, dev, host)) return 1;
    if (run(m, 64, dev, host)) return 1;
    printf("launch %d: block0..7 ->", rep);
    for (int b = 0; b < 8; b++) printf(" %u", host[2 * b] & 15);
    printf("\n");
  }
  CK(hipFree(dev));
  return 0;
}
