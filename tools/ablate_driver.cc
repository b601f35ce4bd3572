// ablate_driver.cc -- times lsbm_crc32c_fixed_dev from several builds of the
// library (dlopen) on the same 4 GiB batch.  Diagnostic tool (tools/ablate.sh).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef int (*fixed_fn)(const void*, uint64_t, uint64_t, uint64_t, const uint32_t*, uint32_t*,
                        uint32_t, void*);
typedef int (*fill_fn)(void*, uint64_t, uint64_t, void*);

int main(int argc, char** argv) {
  const uint64_t L = 4096;
  const uint64_t n_max = getenv("ABL_NMAX") ? strtoull(getenv("ABL_NMAX"), 0, 10) : (1ull << 20);
  uint64_t n = n_max;
  uint8_t* d;
  uint32_t *out, *ref;
  if (hipMalloc(&d, L * n) != hipSuccess || hipMalloc(&out, n * 4) != hipSuccess ||
      hipMalloc(&ref, n * 4) != hipSuccess)
    return 1;
  if (getenv("ABL_SWEEP")) {  // one library, batch-size sweep: fixed overhead
    void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    fixed_fn f = (fixed_fn)dlsym(h, "lsbm_crc32c_fixed_dev");
    fill_fn fill = (fill_fn)dlsym(h, "lsbm_fill_splitmix64_dev");
    fill(d, L * n_max, 0x5EED0000, nullptr);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (uint64_t nn : {8192ull, 65536ull, 262144ull, 1ull << 20, 1ull << 21, 1ull << 22, 1ull << 23}) {
      if (nn > n_max) break;
      for (int i = 0; i < 3; i++) f(d, L, L, nn, nullptr, out, 0, nullptr);
      std::vector<float> ms;
      for (int i = 0; i < 11; i++) {
        hipEventRecord(a, nullptr);
        f(d, L, L, nn, nullptr, out, 0, nullptr);
        hipEventRecord(b, nullptr);
        hipEventSynchronize(b);
        float t;
        hipEventElapsedTime(&t, a, b);
        ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      printf("%s n=%8llu  %.4f ms  %.1f GB/s\n", argv[1], (unsigned long long)nn, ms[5],
             L * nn / (ms[5] * 1e-3) / 1e9);
    }
    return 0;
  }
  // Interleaved A/B: every round launches each variant once, so clock and
  // thermal drift hit all variants alike; report medians over rounds.
  const int nv = argc - 1;
  std::vector<fixed_fn> fns(nv);
  for (int v = 0; v < nv; v++) {
    void* h = dlopen(argv[v + 1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      printf("%s: %s\n", argv[v + 1], dlerror());
      return 1;
    }
    fns[v] = (fixed_fn)dlsym(h, "lsbm_crc32c_fixed_dev");
    if (v == 0) ((fill_fn)dlsym(h, "lsbm_fill_splitmix64_dev"))(d, L * n, 0x5EED0000, nullptr);
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<std::vector<float>> ms(nv);
  std::vector<bool> same(nv, true);
  std::vector<uint32_t> h1(n), h2(n);
  for (int round = -3; round < 40; round++) {
    for (int v = 0; v < nv; v++) {
      hipEventRecord(a, nullptr);
      fns[v](d, L, L, n, nullptr, out, 0, nullptr);
      hipEventRecord(b, nullptr);
      hipEventSynchronize(b);
      float t;
      hipEventElapsedTime(&t, a, b);
      if (round >= 0) ms[v].push_back(t);
      if (round == 0) {
        if (v == 0) hipMemcpy(ref, out, n * 4, hipMemcpyDeviceToDevice);
        hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(h2.data(), ref, n * 4, hipMemcpyDeviceToHost);
        same[v] = h1 == h2;
      }
    }
  }
  for (int v = 0; v < nv; v++) {
    std::sort(ms[v].begin(), ms[v].end());
    const float med = ms[v][ms[v].size() / 2];
    printf("%-36s median %.4f ms  %.1f GB/s  min %.4f  (%s)\n", argv[v + 1], med,
           L * n / (med * 1e-3) / 1e9, ms[v][0], same[v] ? "same result" : "differs");
  }
  return 0;
}
