// include/lsbm/table_checksum.h -- C++ host API for lsbm's table/ layer:
// batched SSTable block-trailer seal and verify over a host file image.
//
// Mirrors, for a whole batch of blocks, what the reference does per block:
//   TableBuilder::WriteRawBlock (table/table_builder.cc:237-255)
//       trailer = [type][EncodeFixed32(Mask(Extend(Value(block), &type, 1)))]
//   ReadBlock with ReadOptions::verify_checksums (table/format.cc:95-103)
//       Unmask(DecodeFixed32(data + n + 1)) == Value(data, n + 1)
//       else Status::Corruption("block checksum mismatch")
// Sits on top of the C ABI (include/lsbm_crc32c.h); all CRC work runs on the
// GPU.  No HIP types in this header.
#ifndef LSBM_TABLE_CHECKSUM_H_
#define LSBM_TABLE_CHECKSUM_H_

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "lsbm/status.h"

namespace lsbm {

// table/format.h:22-50 (offset and size of a block inside a table file).
struct BlockHandle {
  uint64_t offset;
  uint64_t size;
};

// include/leveldb/options.h:24-29
enum CompressionType : uint8_t { kNoCompression = 0x0, kSnappyCompression = 0x1 };

// table/format.h:84
static const size_t kBlockTrailerSize = 5;

// Lay n blocks of the given sizes back to back, each followed by its 5-byte
// trailer (offset += size + kBlockTrailerSize, table/table_builder.cc:251).
// Returns the handles; *file_size receives the total image size.
std::vector<BlockHandle> LayoutBlocks(const std::vector<uint64_t>& sizes, uint64_t* file_size);

// Batched WriteRawBlock: for every handle, writes the trailer at
// file[offset + size, offset + size + 5) with type = types[i].  A handle
// whose size + 5 bytes leave the image is Corruption("truncated block read")
// (table/format.cc:88-91) and nothing is written.
Status SealBlocks(int device, char* file, size_t file_size, const BlockHandle* handles,
                  const uint8_t* types, size_t n);

// How an image's memory may be page-locked for a call (VerifyBlocks,
// VerifyTables; SealBlocks / SealTables write their images, so those are
// writable by definition):
//  * kImagesWritable -- writable memory the caller owns, as lsbm's ReadBlock
//    has it: it preads every block into `new char[n + kBlockTrailerSize]`
//    (table/format.cc:79-82; lsbm reads no table through mmap,
//    util/env_posix.cc:329-330).  A small job's image is page-locked for the
//    call and DMA-ed in place, as the seal's is (no staging copy);
//  * kImagesReadOnly -- possibly a read-only mapping (an mmap'd table file),
//    which must not be pinned for writing (that could copy a private
//    mapping's pages out of the page cache): staged through pinned buffers
//    unless the caller page-locked it.
// The caller states it; it is never inferred from the pointer's constness.
enum ImageMemory : uint8_t { kImagesReadOnly = 0, kImagesWritable = 1 };

// Batched ReadBlock verify.  ok (optional) receives one flag per block.
// Returns Corruption("block checksum mismatch") if any block fails, and
// Corruption("truncated block read") for a handle past the image.
Status VerifyBlocks(int device, const char* file, size_t file_size, const BlockHandle* handles,
                    size_t n, std::vector<uint8_t>* ok, ImageMemory memory = kImagesReadOnly);

// One table file image in host memory: its blocks and, for sealing, their
// CompressionType bytes.
struct TableImage {
  char* file;
  size_t file_size;
  const BlockHandle* handles;
  const uint8_t* types;  // SealTables only
  size_t n;
};

// SealBlocks / VerifyBlocks over many tables at once (the output tables of a
// compaction, lsbm/db_impl.cc:843-892): the blocks of all of them stream
// through one pipeline (64 MiB chunks, three in flight: host copy, PCIe and
// the kernel overlap), and only 4 B (seal) or 1 B (verify) per block comes
// back from the device.  VerifyTables' ok holds the tables' flags one after
// the other.  A page-locked image (hipHostMalloc / hipHostRegister) is DMA-ed
// in place; a pageable one is copied into pinned staging first.
// VerifyTables' images are read-only memory unless `memory` says they are
// writable heap buffers (ImageMemory above).
Status SealTables(int device, const TableImage* tables, size_t count);
Status VerifyTables(int device, const TableImage* tables, size_t count, std::vector<uint8_t>* ok);
Status VerifyTables(int device, const TableImage* tables, size_t count, std::vector<uint8_t>* ok,
                    ImageMemory memory);

}  // namespace lsbm

#endif  // LSBM_TABLE_CHECKSUM_H_
