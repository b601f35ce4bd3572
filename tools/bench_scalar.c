/* bench_scalar.c -- Level 1 of INTEGRATION.md, measured: the per-call scalar
 * crc32c::Value a relinked lsbm gets from liblsbm_crc32c.so (the x86 crc32
 * instruction, three interleaved 1 KiB streams; lsbm_amd/csrc/crc32c_host.cc)
 * against the reference's own util/crc32c.cc (slice-by-4, oracle/_ref, built
 * from /root/reference), one core, at the sizes lsbm checksums one at a time:
 * a 100-B record, a 1,270-B WAL record (db_bench's mean), a 4,119-B SSTable
 * block || type, a 32 KiB log block and 64 KiB.  Both libraries are dlopen'ed
 * RTLD_LOCAL (each exports leveldb::crc32c::Extend); results are compared.
 *
 *   build: gcc -O2 -o build/bench_scalar tools/bench_scalar.c -ldl
 *   run:   build/bench_scalar lsbm_amd/liblsbm_crc32c.so oracle/_ref/libref_crc32c.so
 * prints one JSON line per size. */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef uint32_t (*value_fn)(const char*, size_t);

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ns per call of f over `buf` rotated through 64 offsets, ~0.25 s */
static double ns_per_call(value_fn f, const char* buf, size_t n, uint32_t* sink) {
  uint64_t calls = 0;
  uint32_t acc = 0;
  const double t0 = now();
  double t = t0;
  while (t - t0 < 0.25) {
    for (int k = 0; k < 256; k++) acc ^= f(buf + (k & 63), n);
    calls += 256;
    t = now();
  }
  *sink ^= acc;
  return (t - t0) * 1e9 / calls;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s liblsbm_crc32c.so libref_crc32c.so\n", argv[0]);
    return 2;
  }
  void* a = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  void* b = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
  if (!a || !b) {
    fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  value_fn ours = (value_fn)dlsym(a, "lsbm_crc32c_value");
  value_fn ref = (value_fn)dlsym(b, "ref_value");
  if (!ours || !ref) {
    fprintf(stderr, "dlsym failed\n");
    return 2;
  }
  const size_t sizes[] = {100, 1270, 4119, 32768, 65536};
  char* buf = malloc(65536 + 64);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < 65536 + 64; i++) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    buf[i] = (char)x;
  }
  uint32_t sink = 0;
  int bad = 0;
  for (int k = 0; k < 64; k++)
    for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++) bad += ours(buf + k, sizes[s]) != ref(buf + k, sizes[s]);
  for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++) {
    const size_t n = sizes[s];
    const double r = ns_per_call(ref, buf, n, &sink), o = ns_per_call(ours, buf, n, &sink);
    printf("{\"bytes\": %zu, \"reference_ns\": %.1f, \"reference_GBps\": %.2f, \"lsbm_ns\": %.1f, \"lsbm_GBps\": %.2f, "
           "\"speedup\": %.1f, \"mismatches\": %d}\n",
           n, r, n / r, o, n / o, r / o, bad);
  }
  return (int)(sink == 0xFFFFFFFFu) + (bad != 0);
}
