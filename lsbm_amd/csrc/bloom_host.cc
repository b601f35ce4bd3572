// bloom_host.cc -- the scalar half of include/lsbm_bloom.h and
// include/util/hash.h, on the host CPU: the reference's out-of-line
// leveldb::Hash (util/hash.cc:18-49, exported under its mangled name so
// util/bloom.cc and the block cache link unchanged) and the filter-size /
// probe-count rules of BloomFilterPolicy.  Batches never come here: they run
// on the GPU through bloom_engine.cc.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/lsbm_bloom.h"
#include "../../include/util/hash.h"

namespace leveldb {

__attribute__((visibility("default"))) uint32_t Hash(const char* data, size_t n, uint32_t seed) {
  constexpr uint32_t m = 0xc6a4a793u;
  uint32_t h = seed ^ (uint32_t)(n * m);
  const unsigned char* p = reinterpret_cast<const unsigned char*>(data);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {  // DecodeFixed32: little-endian word
    const uint32_t w = (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) |
                       ((uint32_t)p[i + 3] << 24);
    h = (h + w) * m;
    h ^= h >> 16;
  }
  // the reference adds `char` values here: signed on x86 (util/hash.cc:35-47)
  switch (n - i) {
    case 3:
      h += (uint32_t)(int32_t)(signed char)p[i + 2] << 16;
      [[fallthrough]];
    case 2:
      h += (uint32_t)(int32_t)(signed char)p[i + 1] << 8;
      [[fallthrough]];
    case 1:
      h += (uint32_t)(int32_t)(signed char)p[i];
      h *= m;
      h ^= h >> 24;
      break;
    default:
      break;
  }
  return h;
}

}  // namespace leveldb

extern "C" {

__attribute__((visibility("default"))) uint32_t lsbm_bloom_hash(const char* data, size_t n,
                                                                uint32_t seed) {
  return leveldb::Hash(data, n, seed);
}

__attribute__((visibility("default"))) uint64_t lsbm_bloom_filter_bytes(uint64_t n_keys,
                                                                        int bits_per_key) {
  if (bits_per_key < 0) return 0;
  uint64_t bits = n_keys * (uint64_t)bits_per_key;  // util/bloom.cc:39-46
  if (bits < 64) bits = 64;
  return (bits + 7) / 8 + 1;  // + the k byte (:50)
}

__attribute__((visibility("default"))) uint32_t lsbm_bloom_k(int bits_per_key) {
  size_t k = (size_t)(bits_per_key * 0.69);  // util/bloom.cc:27-30 (0.69 ~ ln 2, rounded down)
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return (uint32_t)k;
}

__attribute__((visibility("default"))) uint64_t lsbm_bloom_k_probe(int bits_per_key,
                                                                   int bloom_bits_use) {
  // include/leveldb/params.h:65-71: not clamped, so 0 probes (always "may match") is possible
  const int raw =
      (bloom_bits_use < bits_per_key && bloom_bits_use > 0) ? bloom_bits_use : bits_per_key;
  return raw > 0 ? (uint64_t)(raw * 0.69) : 0;
}

}  // extern "C"
