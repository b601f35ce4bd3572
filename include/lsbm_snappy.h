/*
 * lsbm_snappy.h -- C ABI of the MI355X (gfx950) batched snappy block codec for
 * lsbm's SSTable blocks.  Implemented by lsbm_amd/liblsbm_crc32c.so, with the
 * conventions of include/lsbm_crc32c.h: extern "C", plain pointers and sizes,
 * LSBM_* status codes, never throws; `_dev` calls take device pointers and an
 * explicit stream (`void*` hipStream_t) and only enqueue.
 *
 * Reference interfaces replaced (lsbm = tengdj/lsbm), each batched:
 *   port/port_posix.h:119-129  Snappy_Compress (snappy::MaxCompressedLength +
 *                              snappy::RawCompress), called per block by
 *                              TableBuilder::WriteBlock (table/table_builder.cc:
 *                              181-193) -> lsbm_snappy_max_compressed_length,
 *                              lsbm_snappy_compress_dev
 *   port/port_posix.h:131-139  Snappy_GetUncompressedLength, called by ReadBlock
 *                              (table/format.cc:125-128)
 *                              -> lsbm_snappy_uncompressed_length_dev
 *   port/port_posix.h:141-148  Snappy_Uncompress (snappy::RawUncompress), called
 *                              by ReadBlock (table/format.cc:129-134)
 *                              -> lsbm_snappy_uncompress_dev
 * Output is byte-identical to libsnappy >= 1.1.10 (the version pinned by
 * tests/golden/snappy_fixture.json); any snappy decoder reads it.
 */
#ifndef LSBM_SNAPPY_H_
#define LSBM_SNAPPY_H_

#include <stddef.h>
#include <stdint.h>

#include "lsbm_crc32c.h" /* LSBM_* status codes */

#ifdef __cplusplus
extern "C" {
#endif

/* snappy::MaxCompressedLength: 32 + n + n/6 (host, scalar). */
uint64_t lsbm_snappy_max_compressed_length(uint64_t n);

/* Compress block i = d_base[d_offsets[i], d_offsets[i+1]) (offsets: n+1
 * entries) into d_out + d_out_offsets[i], which must have room for
 * lsbm_snappy_max_compressed_length(length) bytes; d_out_len[i] = compressed
 * size (UINT64_MAX for a block of 2^32 - 1 bytes or more, which snappy's
 * 32-bit preamble cannot describe). */
int lsbm_snappy_compress_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                             uint8_t* d_out, const uint64_t* d_out_offsets, uint64_t* d_out_len,
                             void* stream);

/* snappy::GetUncompressedLength of block i: d_ok[i] = 1 and d_ulen[i] = the
 * preamble's length, or d_ok[i] = 0 and d_ulen[i] = 0. */
int lsbm_snappy_uncompressed_length_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                                        uint64_t* d_ulen, uint8_t* d_ok, void* stream);

/* snappy::RawUncompress of block i into d_out[d_out_offsets[i],
 * d_out_offsets[i+1]) (n+1 entries; a capacity below the block's preamble
 * length fails the block).  d_ok[i] = 1 on success, 0 where RawUncompress
 * returns false (ReadBlock's "corrupted compressed block contents"); failures
 * are added to *d_n_bad when it is non-null.  The bytes of a failed block's
 * output range are unspecified. */
int lsbm_snappy_uncompress_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n,
                               uint8_t* d_out, const uint64_t* d_out_offsets, uint8_t* d_ok,
                               uint32_t* d_n_bad, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* LSBM_SNAPPY_H_ */
