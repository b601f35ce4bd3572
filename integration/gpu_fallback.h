// integration/gpu_fallback.h -- what the GPU table ends do when the device
// cannot do its part: the block CRCs on the CPU, as the reference computes
// them, so that a GPU problem never changes a table's bytes or a read's
// verdict.
//
// Why: in the reference, WriteRawBlock's checksum cannot fail -- it is pure
// CPU work, and only the file Append can (table/table_builder.cc:243-250).  A
// compaction error in lsbm is sticky: RecordBackgroundError sets bg_error_
// (lsbm/db_impl.cc:567-573) and every later write returns it (:1452-1454).  So
// a transient device error (no device, a HIP error, a staging allocation
// failure) must not surface as a builder or reader error; the trailers are
// then computed here with the library's own scalar crc32c::Extend
// (lsbm_amd/csrc/crc32c_host.cc, the x86 crc32 instruction) and the table is
// byte-identical.  Likewise ReadBlock's check (table/format.cc:88-103) for the
// read side.  Nothing here is test code: it is the product's own slow path,
// counted so that an operator sees it (LSBM_TABLE_STATS).
#ifndef LSBM_INTEGRATION_GPU_FALLBACK_H_
#define LSBM_INTEGRATION_GPU_FALLBACK_H_

#include <stddef.h>
#include <stdint.h>

#include <atomic>

#include "leveldb/status.h"
#include "lsbm/table_checksum.h"
#include "util/coding.h"
#include "util/crc32c.h"

namespace leveldb {

// Process-wide counts of GPU calls that fell back to the CPU.
struct GpuFallbackCounts {
  std::atomic<uint64_t> seals{0};     // GpuTableBuilder::Finish: trailers sealed here
  std::atomic<uint64_t> verifies{0};  // OpenVerifiedTable: data blocks checked here
};
inline GpuFallbackCounts& GpuFallbacks() {
  static GpuFallbackCounts c;
  return c;
}

// WriteRawBlock's trailer for every block (table/table_builder.cc:243-249):
// [type][EncodeFixed32(Mask(Extend(Value(block), &type, 1)))] at
// image[offset + size].  The handles are the builder's own, inside the image.
inline void SealTrailersOnHost(char* image, const lsbm::BlockHandle* handles, const uint8_t* types, size_t n) {
  for (size_t i = 0; i < n; i++) {
    char* block = image + handles[i].offset;
    char* trailer = block + handles[i].size;
    trailer[0] = static_cast<char>(types[i]);
    uint32_t crc = crc32c::Value(block, handles[i].size);
    crc = crc32c::Extend(crc, trailer, 1);  // extend to cover the block type
    EncodeFixed32(trailer + 1, crc32c::Mask(crc));
  }
}

// ReadBlock's check (table/format.cc:88-103) for every block, with
// lsbm::VerifyBlocks' statuses: "truncated block read" when a handle's
// n + 5 bytes leave the image (checked for all handles first, as the GPU
// layer does), else "block checksum mismatch" when any stored crc differs.
inline Status VerifyBlocksOnHost(const char* image, uint64_t size, const lsbm::BlockHandle* handles, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const lsbm::BlockHandle& h = handles[i];
    if (h.offset > size || h.size > size - h.offset || size - h.offset - h.size < lsbm::kBlockTrailerSize)
      return Status::Corruption("truncated block read");
  }
  bool bad = false;
  for (size_t i = 0; i < n; i++) {
    const char* data = image + handles[i].offset;
    const size_t len = handles[i].size;
    const uint32_t stored = crc32c::Unmask(DecodeFixed32(data + len + 1));
    bad = bad || crc32c::Value(data, len + 1) != stored;
  }
  return bad ? Status::Corruption("block checksum mismatch") : Status::OK();
}

}  // namespace leveldb

#endif  // LSBM_INTEGRATION_GPU_FALLBACK_H_
