// tools/probe_pinned_alloc.cc -- does pinned allocation scale with threads?
// 4 x 80 MiB hipHostMalloc (+ the same of hipMalloc), one after another and
// from 4 threads at once (a session's first big job grows 4 stages; DESIGN.md
// section 7).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <thread>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  const size_t n = 80u << 20;
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 1;
  for (int round = 0; round < 3; round++) {
    void* h[4];
    void* d[4];
    auto t = std::chrono::steady_clock::now();
    for (int i = 0; i < 4; i++)
      if (hipHostMalloc(&h[i], n, hipHostMallocDefault) != hipSuccess || hipMalloc(&d[i], n) != hipSuccess) return 1;
    const double seq = ms_since(t);
    for (int i = 0; i < 4; i++) hipHostFree(h[i]), hipFree(d[i]);
    t = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    bool bad = false;
    for (int i = 0; i < 4; i++)
      th.emplace_back([&, i] {
        (void)hipSetDevice(0);
        if (hipHostMalloc(&h[i], n, hipHostMallocDefault) != hipSuccess || hipMalloc(&d[i], n) != hipSuccess) bad = true;
      });
    for (auto& x : th) x.join();
    const double par = ms_since(t);
    if (bad) return 1;
    for (int i = 0; i < 4; i++) hipHostFree(h[i]), hipFree(d[i]);
    printf("{\"round\": %d, \"sequential_ms\": %.2f, \"four_threads_ms\": %.2f}\n", round, seq, par);
  }
  return 0;
}
