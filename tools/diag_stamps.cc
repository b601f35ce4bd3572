// diag_stamps.cc -- per-wave timeline of one crc32c_fixed_kernel launch from a
// -DLSBM_DIAG_STAMPS build (s_memrealtime, 100 MHz).  Diagnostic tool.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef int (*fixed_fn)(const void*, uint64_t, uint64_t, uint64_t, const uint32_t*, uint32_t*,
                        uint32_t, void*);
typedef int (*fill_fn)(void*, uint64_t, uint64_t, void*);
typedef int (*stamps_fn)(uint64_t*, int);

int main(int argc, char** argv) {
  const uint64_t L = 4096, n = 1 << 20;
  void* h = dlopen(argv[1], RTLD_NOW);
  if (!h) { printf("%s\n", dlerror()); return 1; }
  fixed_fn f = (fixed_fn)dlsym(h, "lsbm_crc32c_fixed_dev");
  fill_fn fill = (fill_fn)dlsym(h, "lsbm_fill_splitmix64_dev");
  stamps_fn st = (stamps_fn)dlsym(h, "lsbm_diag_stamps");
  uint8_t* d; uint32_t* out;
  hipMalloc(&d, L * n); hipMalloc(&out, n * 4);
  fill(d, L * n, 0x5EED0000, nullptr);
  for (int i = 0; i < 10; i++) f(d, L, L, n, nullptr, out, 0, nullptr);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 3; rep++) {
    f(d, L, L, n, nullptr, out, 0, nullptr);
    hipDeviceSynchronize();
    std::vector<uint64_t> s(4 * 65536);
    st(s.data(), 0);
    const int nw = 4096;
    uint64_t t0 = ~0ull, tmax = 0;
    for (int w = 0; w < nw; w++) { t0 = std::min(t0, s[w]); tmax = std::max(tmax, s[2 * 65536 + w]); }
    std::vector<double> st0, st1, en;
    std::vector<double> xe(8, 0); std::vector<int> xc(8, 0);
    for (int w = 0; w < nw; w++) {
      st0.push_back((s[w] - t0) * 0.01); st1.push_back((s[65536 + w] - t0) * 0.01);
      en.push_back((s[2 * 65536 + w] - t0) * 0.01);
      int x = (int)s[3 * 65536 + w] & 7; xe[x] += en.back(); xc[x]++;
    }
    auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    printf("rep %d (us): start p0/p50/p100 %.1f/%.1f/%.1f  tables-ready p50/p100 %.1f/%.1f  end p0/p10/p50/p90/p100 %.1f/%.1f/%.1f/%.1f/%.1f\n", rep,
           pct(st0, 0), pct(st0, .5), pct(st0, 1), pct(st1, .5), pct(st1, 1), pct(en, 0), pct(en, .1), pct(en, .5), pct(en, .9), pct(en, 1));
    printf("   mean end per XCC:");
    for (int x = 0; x < 8; x++) printf(" %.1f(%d)", xc[x] ? xe[x] / xc[x] : 0, xc[x]);
    printf("\n");
  }
  return 0;
}
