// bloom_types.h -- argument blocks shared by bloom_engine.cc (host) and
// bloom_kernels.hip (device).  Plain C++, no HIP headers.
#pragma once
#include <stdint.h>

// Diagnostic A/B macros that make a build compute wrong results on purpose
// (results not stored, stored CRCs rewritten, bloom probes not set) are
// refused unless the build also says it is a diagnostic one: such a library
// is only ever written under build/ab/ (tools/build_variant.sh), never the
// product lsbm_amd/liblsbm_crc32c.so.
#if (defined(LSBM_DIAG_NO_STORE) || defined(LSBM_DIAG_VERIFY_WRITEBACK) || \
     defined(LSBM_DIAG_NO_PROBE_WRITES) || defined(LSBM_DIAG_NO_FILTER_LOADS)) && !defined(LSBM_DIAG_BUILD)
#error "LSBM_DIAG_* result-changing macros need LSBM_DIAG_BUILD (A/B variant builds only)"
#endif

namespace lsbm {

constexpr int kBloomThreads = 256;                 // 4 waves per workgroup
constexpr int kBloomWaves = kBloomThreads / 64;
constexpr uint32_t kBloomWindowBytes = 4096;       // filter bytes a wave holds in LDS at once (build_one)
constexpr uint32_t kBloomWindowWords = kBloomWindowBytes / 4;
constexpr uint32_t kBloomRegionWords = 1280;       // a wave's LDS: a packed group's filters + key staging
constexpr uint32_t kBloomGroup = 32;                // filters a wave takes at a time (<= 64)
static_assert(kBloomRegionWords >= kBloomWindowWords + 1, "build_one's window + pad word");

struct BloomBuildArgs {
  const uint8_t* keys;
  const uint64_t* key_offsets;   // key i = keys[off[i], off[i+1] - strip)
  const uint64_t* filter_first;  // n_filters + 1
  const uint64_t* filter_out;    // n_filters byte offsets into out
  uint8_t* out;
  uint64_t n_filters;
  uint64_t bits_per_key;         // size_t bits_per_key_ (util/bloom.cc:19)
  uint32_t strip;
  uint32_t k;                    // k_ (util/bloom.cc:27-30)
};

enum BloomProbeMode : uint32_t {
  kProbeFilter = 0,       // handles name one filter (BloomFilterPolicy::KeyMayMatch)
  kProbeFilterBlock = 1,  // handles name a filter block (FilterBlockReader::KeyMayMatch)
};

struct BloomProbeArgs {
  const uint8_t* base;           // filters / filter blocks
  const uint64_t* handles;       // {offset, size} per query
  const uint64_t* data_offsets;  // kProbeFilterBlock: data block offset per query
  const uint8_t* keys;
  const uint64_t* key_offsets;
  uint8_t* may;
  uint32_t* n_may;               // nullable
  uint64_t n;
  uint64_t k_use;                // k_use_ (include/leveldb/params.h:65-71)
  uint32_t strip;
  uint32_t mode;
};

}  // namespace lsbm
