// ref_shim.cc -- TEST INFRASTRUCTURE ONLY.  A C-ABI shim that is compiled
// together with the *reference's own* /root/reference/util/crc32c.cc (never
// copied into this repo) into oracle/_ref/libref_crc32c.so, so that golden
// vectors and the optional "reference" CPU baseline come from the reference
// code itself.  Build recipe: oracle/Makefile (target `ref`).
#include <stddef.h>
#include <stdint.h>
#include <pthread.h>
#include "util/crc32c.h"   // resolved against -I/root/reference

extern "C" {

uint32_t ref_extend(uint32_t crc, const char* p, size_t n) {
  return leveldb::crc32c::Extend(crc, p, n);
}
uint32_t ref_value(const char* p, size_t n) { return leveldb::crc32c::Value(p, n); }
uint32_t ref_mask(uint32_t c) { return leveldb::crc32c::Mask(c); }
uint32_t ref_unmask(uint32_t c) { return leveldb::crc32c::Unmask(c); }

struct ref_job { const char* base; uint64_t stride, len, lo, hi; uint32_t* out; };
static void* ref_worker(void* a) {
  ref_job* j = static_cast<ref_job*>(a);
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->out[i] = leveldb::crc32c::Value(j->base + i * j->stride, j->len);
  return nullptr;
}

// crc32c::Value over n fixed-stride blocks on `threads` pthreads.
int ref_batch_fixed_mt(const char* base, uint64_t stride, uint64_t len, uint64_t n,
                       uint32_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  ref_job jobs[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    uint64_t lo = t * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = ref_job{base, stride, len, lo, hi, out};
    if (pthread_create(&tid[t], nullptr, ref_worker, &jobs[t]) != 0) break;
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], nullptr);
  return started == threads ? 0 : -1;
}

// crc32c::Extend(init[i] or 0, base + ext[2i], ext[2i+1]) for n extents, one
// thread: the reference's per-record loop (WriteRawBlock / EmitPhysicalRecord)
// as the config-1 CPU baseline (tools/bench_configs.py).
void ref_batch_extents(const char* base, const uint64_t* ext, const uint32_t* init,
                       uint32_t* out, uint64_t n) {
  for (uint64_t i = 0; i < n; i++)
    out[i] = leveldb::crc32c::Extend(init ? init[i] : 0, base + ext[2 * i], ext[2 * i + 1]);
}

}  // extern "C"
