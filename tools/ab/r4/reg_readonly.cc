// Does hipHostRegister (default flags) accept a read-only mapping, and does a
// DMA from it then work?  Diagnostic for verify's per-call page locks.
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

int main() {
  const size_t n = 16u << 20;
  char path[] = "/tmp/lsbm_ro_XXXXXX";
  const int fd = mkstemp(path);
  char* buf = (char*)malloc(n);
  memset(buf, 'x', n);
  if (write(fd, buf, n) != (ssize_t)n) return 1;
  void* dev = nullptr;
  if (hipMalloc(&dev, n) != hipSuccess) return 1;
  for (int shared = 0; shared < 2; shared++) {
    void* m = mmap(nullptr, n, PROT_READ, shared ? MAP_SHARED : MAP_PRIVATE, fd, 0);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    printf("%s: readOnlySupported=%d\n", shared ? "MAP_SHARED" : "MAP_PRIVATE", prop.hostRegisterReadOnlySupported);
    hipError_t r = hipHostRegister(m, n, hipHostRegisterDefault);
    printf("  register default: %d (%s)\n", (int)r, hipGetErrorString(r));
    (void)hipGetLastError();
    if (r == hipSuccess) {
      hipError_t d = hipMemcpy(dev, m, n, hipMemcpyHostToDevice);
      printf("  dma: %d (%s)\n", (int)d, hipGetErrorString(d));
      (void)hipGetLastError();
      hipStream_t s;
      (void)hipStreamCreate(&s);
      hipError_t d2 = hipMemcpyAsync(dev, m, n, hipMemcpyHostToDevice, s);
      hipError_t d3 = hipStreamSynchronize(s);
      printf("  async dma: %d, sync: %d (%s)\n", (int)d2, (int)d3, hipGetErrorString(d3));
      (void)hipGetLastError();
      (void)hipStreamDestroy(s);
      printf("  unregister: %d\n", (int)hipHostUnregister(m));
    }
    hipError_t r2 = hipHostRegister(m, n, hipHostRegisterReadOnly);
    printf("  register read-only: %d (%s)\n", (int)r2, hipGetErrorString(r2));
    (void)hipGetLastError();
    if (r2 == hipSuccess) printf("  unregister: %d\n", (int)hipHostUnregister(m));
    munmap(m, n);
  }
  close(fd);
  unlink(path);
  printf("done\n");
  return 0;
}
