/*
 * bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker: never shipped,
 * never on the product path).  A plain-C restatement of lsbm's SSTable filter
 * path, step for step:
 *
 *   util/hash.cc:18-49           leveldb::Hash (murmur-like 4-byte steps; the
 *                                byte tail adds SIGNED chars)
 *   util/bloom.cc:13-15          BloomHash = Hash(key, n, 0xbc9f1d34)
 *   util/bloom.cc:24-31          k_ = (size_t)(bits_per_key * 0.69) in [1, 30]
 *   include/leveldb/params.h:65-71  k_use_ = get_bloom_filter_probe_num(), the
 *                                read-side probe count (config::bloom_bits_use,
 *                                common/params.cc:29, default 15)
 *   util/bloom.cc:37-63          CreateFilter
 *   util/bloom.cc:65-89          KeyMayMatch
 *   common/dbformat.cc:105-119   InternalFilterPolicy: ExtractUserKey drops the
 *                                8-byte sequence/type suffix first (strip = 8)
 *   table/filter_block.cc:14-76  FilterBlockBuilder (one filter per 2 KiB of
 *                                block offsets, the offset array, base_lg)
 *   table/filter_block.cc:78-109 FilterBlockReader::KeyMayMatch
 *
 * Pinned by tests/golden/bloom_fixture.json, produced by the reference's own
 * util/hash.cc, util/bloom.cc and table/filter_block.cc compiled in place
 * (oracle/ref_bloom_shim.cc, tests/golden/make_bloom_fixture.py), and by the
 * filter block of a real db_bench SSTable (tests/golden/real_filter.bin).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* util/hash.cc:18-49.  `data` is `const char*` there: every tail byte is a
 * signed char promoted to int before the shift and the add. */
uint32_t bo_hash(const char* data, size_t n, uint32_t seed) {
  const uint32_t m = 0xc6a4a793u;
  const uint32_t r = 24;
  const char* limit = data + n;
  uint32_t h = seed ^ (uint32_t)(n * m);
  while (data + 4 <= limit) {
    const uint32_t w = (uint32_t)(uint8_t)data[0] | ((uint32_t)(uint8_t)data[1] << 8) |
                       ((uint32_t)(uint8_t)data[2] << 16) | ((uint32_t)(uint8_t)data[3] << 24);
    data += 4;
    h += w;
    h *= m;
    h ^= (h >> 16);
  }
  switch (limit - data) {
    case 3:
      h += (uint32_t)(int32_t)(signed char)data[2] << 16;
      /* fall through */
    case 2:
      h += (uint32_t)(int32_t)(signed char)data[1] << 8;
      /* fall through */
    case 1:
      h += (uint32_t)(int32_t)(signed char)data[0];
      h *= m;
      h ^= (h >> r);
      break;
  }
  return h;
}

/* util/bloom.cc:27-30 */
size_t bo_k_build(int bits_per_key) {
  size_t k = (size_t)(bits_per_key * 0.69);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return k;
}

/* include/leveldb/params.h:65-71 (not clamped: 0 probes is possible) */
size_t bo_k_probe(int bits_per_key, int bloom_bits_use) {
  const int raw =
      (bloom_bits_use < bits_per_key && bloom_bits_use > 0) ? bloom_bits_use : bits_per_key;
  return (size_t)(raw * 0.69);
}

/* Bytes CreateFilter appends for n keys: the bit array and the k byte
 * (util/bloom.cc:39-50). */
size_t bo_filter_bytes(size_t n, int bits_per_key) {
  size_t bits = n * (size_t)bits_per_key;
  if (bits < 64) bits = 64;
  return (bits + 7) / 8 + 1;
}

/* util/bloom.cc:37-63 over keys [offs[i], offs[i+1] - strip) of `keys`,
 * written to dst[0, bo_filter_bytes(n)).  Returns that size. */
size_t bo_create_filter(const char* keys, const uint64_t* offs, size_t n, int strip,
                        int bits_per_key, char* dst) {
  const size_t total = bo_filter_bytes(n, bits_per_key);
  const size_t bytes = total - 1;
  const size_t bits = bytes * 8;
  const size_t k = bo_k_build(bits_per_key);
  memset(dst, 0, bytes);
  dst[bytes] = (char)k;
  for (size_t i = 0; i < n; i++) {
    const size_t len = (size_t)(offs[i + 1] - offs[i]) - (size_t)strip;
    uint32_t h = bo_hash(keys + offs[i], len, 0xbc9f1d34u);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (size_t j = 0; j < k; j++) {
      const uint32_t bitpos = (uint32_t)(h % bits);
      dst[bitpos / 8] |= (char)(1 << (bitpos % 8));
      h += delta;
    }
  }
  return total;
}

/* util/bloom.cc:65-89 (after common/dbformat.cc:117-119 when strip = 8). */
int bo_key_may_match(const char* key, size_t n, int strip, const char* filter, size_t len,
                     int bits_per_key, int bloom_bits_use) {
  if (len < 2) return 0;
  const size_t bits = (len - 1) * 8;
  const size_t k_use = bo_k_probe(bits_per_key, bloom_bits_use);
  /* `array[len-1] > k_use_`: a signed char converted to size_t */
  const size_t stored = (size_t)(long)(signed char)filter[len - 1];
  const size_t k = stored > k_use ? k_use : stored;
  if (k > 30) return 1;
  uint32_t h = bo_hash(key, n - (size_t)strip, 0xbc9f1d34u);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (size_t j = 0; j < k; j++) {
    const uint32_t bitpos = (uint32_t)(h % bits);
    if ((filter[bitpos / 8] & (1 << (bitpos % 8))) == 0) return 0;
    h += delta;
  }
  return 1;
}

/* table/filter_block.cc:18-76 for the call sequence
 *     for b in [0, n_blocks): StartBlock(block_start[b]);
 *                             AddKey(key i) for i in [block_first[b], block_first[b+1])
 *     Finish()
 * (TableBuilder: StartBlock(0) in its constructor, table_builder.cc:79-81;
 * AddKey per Add, :129-131; StartBlock(offset) after each data block written,
 * :154-156).  Keys are keys[key_offs[i], key_offs[i+1]).  Writes the block to
 * out when it fits in cap; returns its size (0 on allocation failure). */
size_t bo_filter_block_build(const char* keys, const uint64_t* key_offs, int strip,
                             const uint64_t* block_start, const uint64_t* block_first,
                             size_t n_blocks, int bits_per_key, char* out, size_t cap) {
  size_t size = 0, nfilt = 0, cap_f = 16;
  uint32_t* foffs = (uint32_t*)malloc(cap_f * sizeof(uint32_t));
  if (!foffs) return 0;
  size_t lo = n_blocks ? (size_t)block_first[0] : 0, hi = lo; /* pending keys [lo, hi) */
  for (size_t b = 0; b <= n_blocks; b++) {
    /* b == n_blocks is Finish(): GenerateFilter only if keys are pending */
    const uint64_t filter_index = b < n_blocks ? block_start[b] / 2048 : 0; /* kFilterBase */
    while (b < n_blocks ? filter_index > nfilt : hi > lo) {
      if (nfilt == cap_f) {
        uint32_t* g = (uint32_t*)realloc(foffs, 2 * cap_f * sizeof(uint32_t));
        if (!g) {
          free(foffs);
          return 0;
        }
        foffs = g;
        cap_f *= 2;
      }
      foffs[nfilt++] = (uint32_t)size; /* :56 / :70 */
      if (hi > lo) {
        const size_t fb = bo_filter_bytes(hi - lo, bits_per_key);
        if (size + fb <= cap)
          bo_create_filter(keys, key_offs + lo, hi - lo, strip, bits_per_key, out + size);
        size += fb;
        lo = hi;
      }
    }
    if (b < n_blocks) hi = (size_t)block_first[b + 1];
  }
  const size_t total = size + 4 * nfilt + 5;
  if (total <= cap) { /* :41-49: offsets, array_offset, kFilterBaseLg */
    for (size_t i = 0; i < nfilt; i++) memcpy(out + size + 4 * i, &foffs[i], 4);
    const uint32_t array_offset = (uint32_t)size;
    memcpy(out + size + 4 * nfilt, &array_offset, 4);
    out[total - 1] = 11;
  }
  free(foffs);
  return total;
}

/* table/filter_block.cc:78-109 with the policy's KeyMayMatch.  base_lg is a
 * size_t loaded from a (signed) char; the shift uses it mod 64 as x86-64 does. */
int bo_filter_block_may_match(const char* contents, size_t n, uint64_t block_offset,
                              const char* key, size_t kn, int strip, int bits_per_key,
                              int bloom_bits_use) {
  if (n < 5) return 1; /* no data_: num_ = 0 -> "errors are potential matches" */
  const size_t base_lg = (size_t)(long)(signed char)contents[n - 1];
  uint32_t last_word;
  memcpy(&last_word, contents + n - 5, 4);
  if (last_word > n - 5) return 1;
  const char* offset = contents + last_word;
  const size_t num = (n - 5 - last_word) / 4;
  const uint64_t index = block_offset >> (base_lg & 63);
  if (index < num) {
    uint32_t start, limit;
    memcpy(&start, offset + index * 4, 4);
    memcpy(&limit, offset + index * 4 + 4, 4);
    if (start <= limit && limit <= (size_t)last_word) {
      return bo_key_may_match(key, kn, strip, contents + start, limit - start, bits_per_key,
                              bloom_bits_use);
    } else if (start == limit) {
      return 0;
    }
  }
  return 1;
}
