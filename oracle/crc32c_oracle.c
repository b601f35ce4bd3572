/*
 * crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle), NOT product code.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's library (oracle/liboracle_crc32c.so).  The product path
 * (lsbm_amd/liblsbm_crc32c.so) never links or calls anything here.
 *
 * A plain-C restatement of lsbm's CRC-32C (LevelDB 1.15 util/crc32c.cc):
 *   - tables:   util/crc32c.cc:16-279 (table0_..table3_, slice-by-4).  They are
 *               NOT copied: table0 is generated from the reflected Castagnoli
 *               polynomial 0x82F63B78 and table_k[i] = (table_{k-1}[i] >> 8) ^
 *               table0[table_{k-1}[i] & 0xff].
 *   - Extend:   util/crc32c.cc:286-329 -- pre-inversion (:289), byte steps up to
 *               4-byte alignment of the *address* (:304-313), 16-byte unrolled
 *               STEP4 x4 (:315-317), 4-byte STEP4 (:319-321), byte tail
 *               (:323-325), post-inversion (:328).
 *   - STEP1/STEP4 macros: util/crc32c.cc:291-302.
 *   - LE_LOAD32 / DecodeFixed32: util/crc32c.cc:282-284, util/coding.h:58-70.
 *   - Value / Mask / Unmask / kMaskDelta: util/crc32c.h:20-40.
 *
 * Pinning: tests/test_oracle.py checks this against tests/golden/*.json, which
 * tests/golden/make_golden.py produced by running the reference's own
 * util/crc32c.cc compiled here (oracle/Makefile -> oracle/_ref/).
 *
 * Also holds the byte generator used by the benchmark configs (splitmix64,
 * SURVEY.md 8d) and a pthread batch driver so bench.py can time the CPU
 * baseline on the GPU box's host cores.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_POLY 0x82F63B78u /* reflected Castagnoli, util/crc32c.cc:5-6 */

static uint32_t g_t0[256], g_t1[256], g_t2[256], g_t3[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t r = i;
    for (int b = 0; b < 8; b++) r = (r >> 1) ^ (ORACLE_POLY & (0u - (r & 1u)));
    g_t0[i] = r;
  }
  for (uint32_t i = 0; i < 256; i++) {
    g_t1[i] = (g_t0[i] >> 8) ^ g_t0[g_t0[i] & 0xffu];
    g_t2[i] = (g_t1[i] >> 8) ^ g_t0[g_t1[i] & 0xffu];
    g_t3[i] = (g_t2[i] >> 8) ^ g_t0[g_t2[i] & 0xffu];
  }
}

void oracle_init(void) { pthread_once(&g_once, build_tables); }

/* util/crc32c.cc:282-284 + util/coding.h:58-70: little-endian 32-bit load. */
static inline uint32_t le_load32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

/* util/crc32c.cc:286-329, same control flow step for step. */
uint32_t oracle_extend(uint32_t crc, const uint8_t* p, size_t n) {
  oracle_init();
  const uint8_t* e = p + n;
  uint32_t l = crc ^ 0xffffffffu; /* :289 */
#define O_STEP1()                                  \
  do {                                             \
    l = g_t0[(l ^ *p++) & 0xffu] ^ (l >> 8);       \
  } while (0)
#define O_STEP4()                                                     \
  do {                                                                \
    uint32_t c = l ^ le_load32(p);                                    \
    p += 4;                                                           \
    l = g_t3[c & 0xffu] ^ g_t2[(c >> 8) & 0xffu] ^                    \
        g_t1[(c >> 16) & 0xffu] ^ g_t0[c >> 24];                      \
  } while (0)
  /* :304-313 -- advance to the first 4-byte aligned address (if inside). */
  const uint8_t* x = (const uint8_t*)((((uintptr_t)p) + 3) & ~(uintptr_t)3);
  if (x <= e) {
    while (p != x) O_STEP1();
  }
  while (e - p >= 16) { /* :315-317 */
    O_STEP4(); O_STEP4(); O_STEP4(); O_STEP4();
  }
  while (e - p >= 4) O_STEP4(); /* :319-321 */
  while (p != e) O_STEP1();     /* :323-325 */
#undef O_STEP1
#undef O_STEP4
  return l ^ 0xffffffffu; /* :328 */
}

uint32_t oracle_value(const uint8_t* p, size_t n) { return oracle_extend(0, p, n); }

/* util/crc32c.h:24-40 */
uint32_t oracle_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t oracle_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

void oracle_tables(uint32_t* out1024) {
  oracle_init();
  memcpy(out1024, g_t0, 1024);
  memcpy(out1024 + 256, g_t1, 1024);
  memcpy(out1024 + 512, g_t2, 1024);
  memcpy(out1024 + 768, g_t3, 1024);
}

/* ---- batch drivers (what the GPU batch API computes, done block by block) ---- */

#define ORACLE_FLAG_MASK 1

static inline uint32_t finish(uint32_t crc, int flags) {
  return (flags & ORACLE_FLAG_MASK) ? oracle_mask(crc) : crc;
}

/* Block i = base[offsets[i] .. offsets[i+1]); init may be NULL (Value). */
void oracle_batch_offsets(const uint8_t* base, const uint64_t* offsets, uint64_t n,
                          const uint32_t* init, uint32_t* out, int flags) {
  for (uint64_t i = 0; i < n; i++) {
    uint32_t c0 = init ? init[i] : 0u;
    out[i] = finish(oracle_extend(c0, base + offsets[i], offsets[i + 1] - offsets[i]), flags);
  }
}

/* Block i = base[i*stride .. i*stride+len). */
void oracle_batch_fixed(const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n,
                        const uint32_t* init, uint32_t* out, int flags) {
  for (uint64_t i = 0; i < n; i++) {
    uint32_t c0 = init ? init[i] : 0u;
    out[i] = finish(oracle_extend(c0, base + i * stride, len), flags);
  }
}

typedef struct {
  const uint8_t* base;
  uint64_t stride, len, lo, hi;
  uint32_t* out;
} fixed_job;

static void* fixed_worker(void* arg) {
  fixed_job* j = (fixed_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) j->out[i] = oracle_extend(0, j->base + i * j->stride, j->len);
  return NULL;
}

/* Same as oracle_batch_fixed (init=NULL, flags=0) on `threads` pthreads. */
int oracle_batch_fixed_mt(const uint8_t* base, uint64_t stride, uint64_t len, uint64_t n,
                          uint32_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  oracle_init();
  pthread_t tid[256];
  fixed_job jobs[256];
  uint64_t per = (n + (uint64_t)threads - 1) / (uint64_t)threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    uint64_t lo = (uint64_t)t * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (fixed_job){base, stride, len, lo, hi, out};
    if (pthread_create(&tid[t], NULL, fixed_worker, &jobs[t]) != 0) break;
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
  return started == threads ? 0 : -1;
}

/* Multithreaded drivers for the full-size parity tests (every block of config 4
 * and of a 1M-block SSTable image checked, not a sample).  Both split [0, n)
 * into `threads` equal block ranges; each block goes through oracle_extend
 * (util/crc32c.cc:286-329) exactly as the scalar drivers above do. */
typedef struct {
  const uint8_t* base;
  const uint64_t* offsets; /* offsets: block i = [offsets[i], offsets[i+1]) - base_off */
  const uint8_t* types;    /* sst: NULL for offsets jobs */
  uint64_t base_off, lo, hi;
  uint32_t* out;
} span_job;

static void* offsets_worker(void* arg) {
  span_job* j = (span_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->out[i] = oracle_extend(0, j->base + (j->offsets[i] - j->base_off), j->offsets[i + 1] - j->offsets[i]);
  return NULL;
}

/* table/table_builder.cc:243-249 (WriteRawBlock): the trailer's crc field is
 * Mask(Extend(Value(block), &type, 1)).  offsets holds BlockHandle pairs
 * {offset, size} here (table/format.h:20-47). */
static void* sst_worker(void* arg) {
  span_job* j = (span_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint64_t off = j->offsets[2 * i] - j->base_off, size = j->offsets[2 * i + 1];
    const uint32_t crc = oracle_extend(0, j->base + off, size);
    j->out[i] = oracle_mask(oracle_extend(crc, &j->types[i], 1));
  }
  return NULL;
}

static int run_spans(void* (*fn)(void*), const uint8_t* base, const uint64_t* offsets, const uint8_t* types,
                     uint64_t base_off, uint64_t n, uint32_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  oracle_init();
  pthread_t tid[256];
  span_job jobs[256];
  const uint64_t per = (n + (uint64_t)threads - 1) / (uint64_t)threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    uint64_t lo = (uint64_t)t * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (span_job){base, offsets, types, base_off, lo, hi, out};
    if (pthread_create(&tid[t], NULL, fn, &jobs[t]) != 0) break;
    started++;
  }
  for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
  return started == threads ? 0 : -1;
}

/* oracle_batch_offsets (init=NULL, flags=0) on `threads` pthreads, over a
 * window of the image: base points at image byte base_off, and every block
 * [offsets[i], offsets[i+1]) of the n must lie in the window. */
int oracle_batch_offsets_mt(const uint8_t* base, uint64_t base_off, const uint64_t* offsets, uint64_t n,
                            uint32_t* out, int threads) {
  return run_spans(offsets_worker, base, offsets, NULL, base_off, n, out, threads);
}

/* The masked trailer crc of n SSTable blocks (handles {offset, size}, types
 * per block) on `threads` pthreads, over a window as above. */
int oracle_sst_trailers_mt(const uint8_t* base, uint64_t base_off, const uint64_t* handles, const uint8_t* types,
                           uint64_t n, uint32_t* out, int threads) {
  return run_spans(sst_worker, base, handles, types, base_off, n, out, threads);
}

/* ---- benchmark byte generator: 8-byte word w of a buffer is
 *      splitmix64(seed + w), stored little-endian. ---- */
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* Fill dst[0..nbytes) with the bytes that live at absolute buffer offsets
 * [byte_off, byte_off+nbytes) of the splitmix64 stream for `seed`. */
void oracle_fill_splitmix64(uint8_t* dst, uint64_t byte_off, uint64_t nbytes, uint64_t seed) {
  for (uint64_t k = 0; k < nbytes; k++) {
    uint64_t a = byte_off + k;
    uint64_t w = splitmix64(seed + (a >> 3));
    dst[k] = (uint8_t)(w >> (8 * (a & 7)));
  }
}
