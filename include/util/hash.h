// include/util/hash.h -- drop-in for lsbm's util/hash.h (util/hash.h:13-17).
//
// Same namespace, name and signature, so util/bloom.cc and the cache link
// unchanged against liblsbm_crc32c.so, which exports leveldb::Hash
// (_ZN7leveldb4HashEPKcmj, lsbm_amd/csrc/bloom_host.cc).  Batches of filters
// and lookups go to the GPU through include/lsbm_bloom.h instead.
#ifndef STORAGE_LEVELDB_UTIL_HASH_H_
#define STORAGE_LEVELDB_UTIL_HASH_H_

#include <stddef.h>
#include <stdint.h>

namespace leveldb {

// util/hash.cc:18-49: murmur-like, 4-byte little-endian steps, signed-char tail.
uint32_t Hash(const char* data, size_t n, uint32_t seed);

}  // namespace leveldb

#endif  // STORAGE_LEVELDB_UTIL_HASH_H_
