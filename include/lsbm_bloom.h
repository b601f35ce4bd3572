/*
 * lsbm_bloom.h -- C ABI of the MI355X (gfx950) batched bloom-filter engine for
 * lsbm's SSTable filter blocks.  Implemented by lsbm_amd/liblsbm_crc32c.so,
 * with the conventions of include/lsbm_crc32c.h: extern "C", plain pointers
 * and sizes, LSBM_* status codes, never throws; `_dev` calls take device
 * pointers and an explicit stream (`void*` hipStream_t) and only enqueue.
 *
 * Reference interfaces replaced (lsbm = tengdj/lsbm):
 *   util/hash.cc:18-49          leveldb::Hash -> lsbm_bloom_hash (host, scalar)
 *                               and include/util/hash.h (same C++ API; the
 *                               library exports _ZN7leveldb4HashEPKcmj)
 *   util/bloom.cc:24-31         BloomFilterPolicy's k_ -> lsbm_bloom_k
 *   include/leveldb/params.h:65-71  k_use_ (get_bloom_filter_probe_num with
 *                               config::bloom_bits_use) -> lsbm_bloom_k_probe
 *   util/bloom.cc:37-63         CreateFilter, for many filters in one launch
 *                               -> lsbm_bloom_build_dev
 *   util/bloom.cc:65-89         KeyMayMatch, for many lookups in one launch
 *                               -> lsbm_bloom_may_match_dev
 *   table/filter_block.cc:95-109  FilterBlockReader::KeyMayMatch, batched
 *                               -> lsbm_filter_block_may_match_dev
 *   common/dbformat.cc:105-119  InternalFilterPolicy (drop the 8-byte
 *                               sequence/type suffix first) -> `strip` = 8
 * FilterBlockBuilder (table/filter_block.cc:18-76) is the C++ layer
 * include/lsbm/filter_block.h on top of these.
 */
#ifndef LSBM_BLOOM_H_
#define LSBM_BLOOM_H_

#include <stddef.h>
#include <stdint.h>

#include "lsbm_crc32c.h" /* LSBM_* status codes */

#ifdef __cplusplus
extern "C" {
#endif

#define LSBM_BLOOM_SEED 0xbc9f1d34u     /* util/bloom.cc:14 */
#define LSBM_FILTER_BASE_LG 11          /* table/filter_block.cc:15 (2 KiB) */
#define LSBM_INTERNAL_KEY_SUFFIX 8      /* common/dbformat.h:75-78 */

/* ---- host helpers (scalar, CPU) ---- */
/* util/hash.cc:18-49 (signed-char tail included). */
uint32_t lsbm_bloom_hash(const char* data, size_t n, uint32_t seed);
/* Bytes CreateFilter appends for n_keys keys: the bit array plus one k byte
 * (util/bloom.cc:39-50); 0 if bits_per_key < 0. */
uint64_t lsbm_bloom_filter_bytes(uint64_t n_keys, int bits_per_key);
/* k_ of BloomFilterPolicy(bits_per_key) (util/bloom.cc:27-30). */
uint32_t lsbm_bloom_k(int bits_per_key);
/* k_use_ (include/leveldb/params.h:65-71) for config::bloom_bits_use. */
uint64_t lsbm_bloom_k_probe(int bits_per_key, int bloom_bits_use);

/* ---- device batches ---- */
/* CreateFilter for n_filters filters.  Key i is
 *     d_keys[key_offsets[i], key_offsets[i+1] - strip)
 * (a key shorter than strip hashes as empty).  Filter f holds keys
 * [filter_first[f], filter_first[f+1]) and is written to
 *     d_out[filter_out[f], filter_out[f] + lsbm_bloom_filter_bytes(n_f, bits_per_key))
 * byte for byte as BloomFilterPolicy(bits_per_key)::CreateFilter appends it.
 * Filters must not overlap; bytes of d_out outside them are not written. */
int lsbm_bloom_build_dev(const void* d_keys, const uint64_t* d_key_offsets, uint32_t strip,
                         const uint64_t* d_filter_first, const uint64_t* d_filter_out,
                         uint64_t n_filters, int bits_per_key, uint8_t* d_out, void* stream);

/* KeyMayMatch for n_queries lookups: key q (as above) against the filter
 * d_filters[handles[2q], handles[2q] + handles[2q+1]) of a
 * BloomFilterPolicy(bits_per_key) with config::bloom_bits_use.  d_may[q] = 0/1;
 * the number of 1s is ADDED to *d_n_may when it is not NULL. */
int lsbm_bloom_may_match_dev(const uint8_t* d_filters, const uint64_t* d_filter_handles,
                             const void* d_keys, const uint64_t* d_key_offsets, uint32_t strip,
                             uint64_t n_queries, int bits_per_key, int bloom_bits_use,
                             uint8_t* d_may, uint32_t* d_n_may, void* stream);

/* FilterBlockReader(policy, contents).KeyMayMatch(block_offset, key) for
 * n_queries lookups: contents = d_blocks[handles[2q], + handles[2q+1]) (a
 * filter block as FilterBlockBuilder::Finish wrote it), block_offset =
 * d_data_offsets[q] (the data block's BlockHandle offset, table/table.cc:321).
 * Malformed blocks answer exactly as the reference: "errors are treated as
 * potential matches", empty filters match nothing.  Outputs as above. */
int lsbm_filter_block_may_match_dev(const uint8_t* d_blocks, const uint64_t* d_block_handles,
                                    const uint64_t* d_data_offsets, const void* d_keys,
                                    const uint64_t* d_key_offsets, uint32_t strip,
                                    uint64_t n_queries, int bits_per_key, int bloom_bits_use,
                                    uint8_t* d_may, uint32_t* d_n_may, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* LSBM_BLOOM_H_ */
