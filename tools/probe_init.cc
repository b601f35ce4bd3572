// tools/probe_init.cc -- where a process's first GPU call spends its time:
// the HIP runtime's own start (hipInit + the device's context) against the
// library's device setup on top (lsbm_crc32c_init: its tables, built on the
// host and copied) and the first launch.  DESIGN.md section 7.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

#include "lsbm_crc32c.h"

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  auto t = std::chrono::steady_clock::now();
  if (hipInit(0) != hipSuccess) return 1;
  const double init = ms_since(t);
  t = std::chrono::steady_clock::now();
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 1;
  const double ctx = ms_since(t);
  t = std::chrono::steady_clock::now();
  if (lsbm_crc32c_init(0) != LSBM_OK) return 1;
  const double lib = ms_since(t);
  void* d = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&d, 8 * 4096) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  t = std::chrono::steady_clock::now();
  if (lsbm_crc32c_fixed_dev(d, 4096, 4096, 8, nullptr, out, 0, nullptr) != LSBM_OK) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const double first = ms_since(t);
  t = std::chrono::steady_clock::now();
  if (lsbm_crc32c_fixed_dev(d, 4096, 4096, 8, nullptr, out, 0, nullptr) != LSBM_OK) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const double second = ms_since(t);
  printf("{\"hipInit_ms\": %.3f, \"context_ms\": %.3f, \"lsbm_init_ms\": %.3f, \"first_launch_ms\": %.3f, "
         "\"second_launch_ms\": %.3f}\n", init, ctx, lib, first, second);
  return 0;
}
