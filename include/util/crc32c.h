// include/util/crc32c.h -- drop-in for lsbm's util/crc32c.h (util/crc32c.h:11-43).
//
// Same namespace, names, signatures and semantics, so table/, common/log_*
// and lsbm/ compile and link unchanged against liblsbm_crc32c.so:
//   * Extend   -- out of line, exported with the reference's mangled name
//                 _ZN7leveldb6crc32c6ExtendEjPKcm (lsbm_amd/csrc/crc32c_host.cc)
//   * Value    -- Extend(0, data, n)                       (util/crc32c.h:20-22)
//   * Mask     -- rotate right 15, add kMaskDelta           (util/crc32c.h:24-34)
//   * Unmask   -- its inverse                               (util/crc32c.h:36-40)
// Batches of blocks go to the GPU through include/lsbm_crc32c.h instead.
#ifndef STORAGE_LEVELDB_UTIL_CRC32C_H_
#define STORAGE_LEVELDB_UTIL_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

namespace leveldb {
namespace crc32c {

// crc32c(A || data[0, n)) given init_crc = crc32c(A).
uint32_t Extend(uint32_t init_crc, const char* data, size_t n);

inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;

// Stored CRCs are masked so that a CRC over data that embeds CRCs stays strong.
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

inline uint32_t Unmask(uint32_t masked_crc) {
  const uint32_t r = masked_crc - kMaskDelta;
  return (r >> 17) | (r << 15);
}

}  // namespace crc32c
}  // namespace leveldb

#endif  // STORAGE_LEVELDB_UTIL_CRC32C_H_
