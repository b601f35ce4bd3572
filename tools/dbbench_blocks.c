/* dbbench_blocks.c -- db_bench-shaped SSTable data blocks, fast and
 * deterministic, for tools/bench_snappy.py (the same layout as
 * tests/golden/snappy_inputs.py dbbench_block): BlockBuilder
 * entries (table/block_builder.cc:63-107: restart every 16 entries, varint
 * shared / non-shared / value lengths, key delta, value; then the restart
 * array and its count) over internal keys "user%019d" + 8-byte (seq << 8 | 1)
 * and 100-byte values made of 50 random printable bytes repeated
 * (util/testutil.cc CompressibleString, ratio 0.5).  Blocks close once they
 * reach block_size (4,096 B, util/options.cc:22), so they come out at
 * ~4.1 KB like the db_bench blocks of SURVEY.md 3.5.
 *
 *   size_t dbgen_blocks(uint64_t seed, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offs)
 * writes n blocks back to back (offs[0..n]); returns the bytes needed (out
 * may be NULL to size the buffer).  */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint64_t sm(uint64_t* x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int varint(uint8_t* p, uint32_t v) {
  int n = 0;
  while (v >= 128) {
    p[n++] = (uint8_t)(v | 128);
    v >>= 7;
  }
  p[n++] = (uint8_t)v;
  return n;
}

/* one block into b (>= 8 KiB); returns its length */
static size_t one_block(uint64_t* rng, uint64_t* key, uint8_t* b) {
  uint32_t restarts[64];
  int nr = 0, count = 0;
  size_t len = 0;
  char last[32], cur[32];
  int last_len = 0;
  while (len + 4 * (size_t)(nr + 1) < 4096) {
    int kl = snprintf(cur, sizeof(cur), "user%019llu", (unsigned long long)*key);
    uint64_t tag = ((1 + *key) << 8) | 1;
    memcpy(cur + kl, &tag, 8);
    kl += 8;
    int shared = 0;
    if (count % 16 == 0) {
      restarts[nr++] = (uint32_t)len;
    } else {
      while (shared < last_len && shared < kl && last[shared] == cur[shared]) shared++;
    }
    len += varint(b + len, shared);
    len += varint(b + len, kl - shared);
    len += varint(b + len, 100);
    memcpy(b + len, cur + shared, kl - shared);
    len += kl - shared;
    uint8_t raw[50];
    for (int i = 0; i < 50; i++) raw[i] = (uint8_t)(32 + sm(rng) % 95);
    memcpy(b + len, raw, 50);
    memcpy(b + len + 50, raw, 50);
    len += 100;
    memcpy(last, cur, kl);
    last_len = kl;
    (*key)++;
    count++;
  }
  for (int i = 0; i < nr; i++, len += 4) memcpy(b + len, &restarts[i], 4);
  memcpy(b + len, &nr, 4);
  return len + 4;
}

size_t dbgen_blocks(uint64_t seed, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offs) {
  uint64_t rng = seed, key = seed % 1000000;
  uint8_t tmp[8192];
  size_t pos = 0;
  if (offs) offs[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    size_t l = one_block(&rng, &key, tmp);
    if (out && pos + l <= cap) memcpy(out + pos, tmp, l);
    pos += l;
    if (offs) offs[i + 1] = pos;
  }
  return pos;
}
