// include/lsbm/filter_block.h -- C++ host API for lsbm's SSTable filter
// blocks (table/filter_block.h:20-64) with the bloom work done on the GPU.
//
//   FilterBlockBuilder  same call protocol as the reference's
//                       ((StartBlock AddKey*)* Finish, table/filter_block.h:27-28)
//                       and byte-identical output; the CreateFilter calls that
//                       the reference makes in GenerateFilter
//                       (table/filter_block.cc:52-76) are deferred to Finish,
//                       which computes every filter in one GPU batch
//                       (lsbm_bloom_build_dev).
//   FinishFilterBlocks  Finish for many tables at once (the outputs of one
//                       compaction): one GPU batch for all of them.
//   FilterBlockReader   FilterBlockReader::KeyMayMatch (table/filter_block.cc:95-109)
//                       for a batch of (block offset, key) lookups
//                       (lsbm_filter_block_may_match_dev).
// The policy is BloomFilterPolicy (util/bloom.cc), optionally wrapped in
// InternalFilterPolicy (common/dbformat.cc:105-119) as DBImpl does
// (lsbm/db_impl.cc:110,135).  No HIP types in this header.
#ifndef LSBM_FILTER_BLOCK_H_
#define LSBM_FILTER_BLOCK_H_

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "lsbm/status.h"

namespace lsbm {

struct BloomOptions {
  int bits_per_key = 20;      // NewBloomFilterPolicy(FLAGS_bloom_bits), lsbm/db_bench.cc:100,548
  int bloom_bits_use = 15;    // config::bloom_bits_use, common/params.cc:29 (read side)
  bool internal_keys = true;  // keys carry the 8-byte sequence/type suffix (InternalFilterPolicy)
};

class FilterBlockBuilder {
 public:
  explicit FilterBlockBuilder(const BloomOptions& options);

  void StartBlock(uint64_t block_offset);  // table/filter_block.cc:22-28
  void AddKey(const char* key, size_t n);  // table/filter_block.cc:30-34
  // table/filter_block.cc:36-50: the finished block, every filter computed
  // on `device` in one batch.
  Status Finish(int device, std::string* result);

 private:
  friend Status FinishFilterBlocks(int device, FilterBlockBuilder* const* builders, size_t n,
                                   std::string* results);
  struct Range {
    uint64_t lo, hi;  // keys [lo, hi) of one filter; empty: no filter bytes
  };
  void GenerateFilter();  // table/filter_block.cc:52-76 without the CreateFilter

  BloomOptions options_;
  std::string keys_;              // flattened key contents
  std::vector<uint64_t> starts_;  // start of each key in keys_
  uint64_t pending_;              // first key not yet in a filter
  std::vector<Range> filters_;    // one per entry of the offset array
};

// Finish() of n builders (all with the same bits_per_key and key kind) in one
// GPU batch; results[i] receives builders[i]'s block.
Status FinishFilterBlocks(int device, FilterBlockBuilder* const* builders, size_t n,
                          std::string* results);

class FilterBlockReader {
 public:
  // contents[0, n) as FilterBlockBuilder::Finish produced it; must outlive
  // the reader (table/filter_block.h:54-55).
  FilterBlockReader(const BloomOptions& options, const char* contents, size_t n);

  // may[i] = KeyMayMatch(block_offsets[i], key i) for keys
  // keys[key_offsets[i], key_offsets[i+1]), computed on `device` in one batch.
  Status KeyMayMatch(int device, const uint64_t* block_offsets, const char* keys,
                     const uint64_t* key_offsets, size_t n, std::vector<uint8_t>* may) const;

 private:
  BloomOptions options_;
  const char* contents_;
  size_t size_;
};

}  // namespace lsbm

#endif  // LSBM_FILTER_BLOCK_H_
