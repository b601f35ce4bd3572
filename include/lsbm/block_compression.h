// include/lsbm/block_compression.h -- C++ host API for lsbm's table/ layer:
// batched SSTable block compression and decompression over host buffers.
//
// Mirrors, for a whole batch of blocks, what the reference does per block:
//   TableBuilder::WriteBlock (table/table_builder.cc:176-193)
//       port::Snappy_Compress(raw) and keep it only if
//       compressed.size() < raw.size() - raw.size() / 8, else store raw with
//       type kNoCompression
//   ReadBlock (table/format.cc:104-145), after the trailer check
//       kNoCompression: the bytes as they are
//       kSnappyCompression: Snappy_GetUncompressedLength + Snappy_Uncompress,
//           else Status::Corruption("corrupted compressed block contents")
//       any other type: Status::Corruption("bad block type")
// Sits on top of the C ABI (include/lsbm_snappy.h); all snappy work runs on
// the GPU.  No HIP types in this header.
#ifndef LSBM_BLOCK_COMPRESSION_H_
#define LSBM_BLOCK_COMPRESSION_H_

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "lsbm/status.h"
#include "lsbm/table_checksum.h"  // CompressionType

namespace lsbm {

// Batched WriteBlock compression of n raw blocks raw[offsets[i], offsets[i+1])
// (offsets: n + 1 entries).  Block i's contents to write are
// (*out)[(*out_offsets)[i], (*out_offsets)[i+1]) with type (*types)[i], ready
// for SealBlocks.
Status CompressBlocks(int device, const char* raw, const uint64_t* offsets, size_t n,
                      std::string* out, std::vector<uint64_t>* out_offsets,
                      std::vector<uint8_t>* types);

// Batched ReadBlock decompression of n block contents
// data[offsets[i], offsets[i+1]) with their trailer type bytes.  Block i's
// bytes are (*out)[(*out_offsets)[i], (*out_offsets)[i+1]).  ok (optional)
// receives one flag per block; the returned status is that of the first
// failing block in index order, as reading the blocks in order would report.
Status UncompressBlocks(int device, const char* data, const uint64_t* offsets, const uint8_t* types,
                        size_t n, std::string* out, std::vector<uint64_t>* out_offsets,
                        std::vector<uint8_t>* ok);

}  // namespace lsbm

#endif  // LSBM_BLOCK_COMPRESSION_H_
