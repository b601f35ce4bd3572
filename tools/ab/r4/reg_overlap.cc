// What hipHostRegister does with a range that overlaps a registration the
// caller made (a shared first page, or the range's first half), and what a
// DMA from it and the unregisters then return.  Diagnostic for CallLocks.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

static void* g_dev = nullptr;
static int dma(const void* p, size_t n) {
  hipError_t e = hipMemcpy(g_dev, p, n, hipMemcpyHostToDevice);
  return (int)e;
}

int main() {
  const size_t fs = 4u << 20;
  hipMalloc(&g_dev, fs);
  std::vector<char> big(2 * fs + (64u << 10), 'x');
  char* base = big.data();
  char* mid = base + 70001;
  char* img1 = mid + 16;
  char* img2 = img1 + fs + 8192;
  printf("reg caller [base, mid): %d\n", (int)hipHostRegister(base, mid - base, hipHostRegisterDefault));
  printf("reg caller img2 first half: %d\n", (int)hipHostRegister(img2, fs / 2, hipHostRegisterDefault));
  hipPointerAttribute_t a;
  printf("attr img1 first byte: %d\n", (int)hipPointerGetAttributes(&a, img1));
  (void)hipGetLastError();
  hipError_t r1 = hipHostRegister(img1, fs, hipHostRegisterDefault);
  printf("reg img1 (shares a page): %d\n", (int)r1);
  (void)hipGetLastError();
  if (r1 == hipSuccess) {
    printf("dma img1: %d\n", dma(img1, fs));
    printf("unreg img1: %d\n", (int)hipHostUnregister(img1));
  }
  hipError_t r2 = hipHostRegister(img2, fs, hipHostRegisterDefault);
  printf("reg img2 (half registered): %d\n", (int)r2);
  (void)hipGetLastError();
  if (r2 == hipSuccess) {
    printf("dma img2: %d\n", dma(img2, fs));
    printf("unreg img2 (ours): %d\n", (int)hipHostUnregister(img2));
  }
  printf("dma base range: %d\n", dma(base, mid - base));
  printf("unreg caller img2: %d\n", (int)hipHostUnregister(img2));
  printf("unreg caller base: %d\n", (int)hipHostUnregister(base));
  printf("done\n");
  return 0;
}
