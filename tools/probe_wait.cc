// probe_wait.cc -- where a waiting caller's host CPU goes (round 5): per
// call, the calling thread's CPU (RUSAGE_THREAD) and the process's
// (RUSAGE_SELF) for (a) a 16 MiB H2D copy from pinned memory waited on with a
// plain event, (b) the same with a hipEventBlockingSync event, (c) the same
// with hipStreamSynchronize, and (d) SealBlocks of a 16 MiB table (the
// library's own waits; LSBM_BLOCKING_WAIT decides its events).
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include tools/probe_wait.cc \
//       -Llsbm_amd -llsbm_crc32c -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/lsbm_amd -o build/probe_wait
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

#include <vector>

#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"

static double cpu(int who) {
  struct rusage ru;
  getrusage(who, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}
static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

template <class F>
void phase(const char* what, int reps, F f) {
  for (int i = 0; i < 5; i++) f();
  const double w0 = now(), t0 = cpu(RUSAGE_THREAD), p0 = cpu(RUSAGE_SELF);
  for (int i = 0; i < reps; i++) f();
  const double w = (now() - w0) / reps, t = (cpu(RUSAGE_THREAD) - t0) / reps, p = (cpu(RUSAGE_SELF) - p0) / reps;
  printf("{\"what\": \"%s\", \"wall_ms\": %.3f, \"caller_cpu_ms\": %.3f, \"process_cpu_ms\": %.3f}\n", what, w * 1e3,
         t * 1e3, p * 1e3);
}

int main() {
  const size_t n = 16u << 20;
  void *h = nullptr, *d = nullptr;
  hipStream_t s;
  hipEvent_t plain, blocking;
  if (hipHostMalloc(&h, n, 0) != hipSuccess || hipMalloc(&d, n) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&plain, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&blocking, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
    printf("setup failed\n");
    return 1;
  }
  memset(h, 1, n);
  phase("h2d_16MiB_event_plain", 200, [&] {
    (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
    (void)hipEventRecord(plain, s);
    (void)hipEventSynchronize(plain);
  });
  phase("h2d_16MiB_event_blocking", 200, [&] {
    (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
    (void)hipEventRecord(blocking, s);
    (void)hipEventSynchronize(blocking);
  });
  phase("h2d_16MiB_stream_sync", 200, [&] {
    (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
  });
  phase("h2d_16MiB_query_sleep", 200, [&] {  // polling with sleeps: the floor of a waiting caller
    (void)hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s);
    (void)hipEventRecord(plain, s);
    while (hipEventQuery(plain) == hipErrorNotReady) {
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
    }
  });
  std::vector<uint64_t> sizes(4069, 4118);
  uint64_t fs = 0;
  std::vector<lsbm::BlockHandle> hd = lsbm::LayoutBlocks(sizes, &fs);
  std::vector<char> img(fs, 'x');
  std::vector<uint8_t> ty(sizes.size(), 0);
  phase("seal_16MiB_table", 200, [&] { (void)lsbm::SealBlocks(0, img.data(), img.size(), hd.data(), ty.data(), hd.size()); });
  return 0;
}
