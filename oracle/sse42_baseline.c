/* sse42_baseline.c -- TEST / MEASUREMENT INFRASTRUCTURE, not the oracle.
 *
 * The strongest CPU CRC-32C a host offers: the SSE4.2 `crc32` instruction
 * (reflected polynomial 0x82F63B78, no pre/post inversion), run on three
 * blocks at once so that three independent dependency chains hide the
 * instruction's 3-cycle latency.  SURVEY.md 8(d) asks for such a line beside
 * the reference's own slice-by-4 loop (util/crc32c.cc:286-329), labelled "not
 * reference": lsbm itself never uses it.  bench.py's cpu_baseline reports it
 * as `sse42_not_reference`, cross-checked against the GPU's CRCs.  Results are
 * crc32c::Value of each block (init ~0, final ~0), bit-exact with the oracle.
 */
#include <nmmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

static inline uint32_t tail_bytes(uint32_t l, const uint8_t* p, uint64_t n) {
  for (uint64_t k = 0; k < n; k++) l = _mm_crc32_u8(l, p[k]);
  return l;
}

static uint32_t one(const uint8_t* p, uint64_t n) {
  uint64_t l = 0xffffffffu;
  uint64_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    memcpy(&w, p + k, 8);
    l = _mm_crc32_u64(l, w);
  }
  return ~tail_bytes((uint32_t)l, p + k, n - k);
}

/* blocks i, i+1, i+2 interleaved */
static void three(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint64_t n, uint32_t* out) {
  uint64_t la = 0xffffffffu, lb = 0xffffffffu, lc = 0xffffffffu;
  uint64_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t wa, wb, wc;
    memcpy(&wa, a + k, 8);
    memcpy(&wb, b + k, 8);
    memcpy(&wc, c + k, 8);
    la = _mm_crc32_u64(la, wa);
    lb = _mm_crc32_u64(lb, wb);
    lc = _mm_crc32_u64(lc, wc);
  }
  out[0] = ~tail_bytes((uint32_t)la, a + k, n - k);
  out[1] = ~tail_bytes((uint32_t)lb, b + k, n - k);
  out[2] = ~tail_bytes((uint32_t)lc, c + k, n - k);
}

typedef struct {
  const uint8_t* base;
  uint64_t stride, len, lo, hi;
  uint32_t* out;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  uint64_t i = j->lo;
  for (; i + 3 <= j->hi; i += 3)
    three(j->base + i * j->stride, j->base + (i + 1) * j->stride, j->base + (i + 2) * j->stride, j->len,
          j->out + i);
  for (; i < j->hi; i++) j->out[i] = one(j->base + i * j->stride, j->len);
  return NULL;
}

/* crc32c::Value of n fixed-stride blocks on `threads` pthreads; 0 on success. */
int sse42_batch_fixed_mt(const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n, uint32_t* out,
                         int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job jobs[256];
  uint64_t per = (n + (uint64_t)threads - 1) / (uint64_t)threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    uint64_t lo = (uint64_t)t * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (job){base, stride, len, lo, hi, out};
    if (pthread_create(&tid[t], NULL, worker, &jobs[t]) != 0) break;
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
  return started == threads ? 0 : -1;
}
