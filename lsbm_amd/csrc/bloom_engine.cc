// bloom_engine.cc -- the device entry points of include/lsbm_bloom.h.
//
// Validates arguments, sizes the grid and launches bloom_kernels.hip on the
// caller's stream.  Never computes a batch on the CPU: without a usable
// device every entry point returns LSBM_ERR_NO_DEVICE.
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/lsbm_bloom.h"
#include "bloom_types.h"
#include "engine_internal.h"

namespace lsbm {

// launchers (bloom_kernels.hip)
hipError_t launch_bloom_build(const BloomBuildArgs& a, int grid, hipStream_t stream);
hipError_t launch_bloom_probe(const BloomProbeArgs& a, int grid, hipStream_t stream);
int bloom_build_blocks_per_cu();
int bloom_probe_blocks_per_cu(uint32_t mode);

namespace {

int grid_for(int cus, uint64_t items, uint64_t per_wg, uint64_t wgs_per_cu) {
  const uint64_t wgs = (items + per_wg - 1) / per_wg;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(wgs, (uint64_t)cus * wgs_per_cu));
}

int probe(const uint8_t* base, const uint64_t* handles, const uint64_t* data_offsets,
          const void* keys, const uint64_t* key_offsets, uint32_t strip, uint64_t n,
          int bits_per_key, int bloom_bits_use, uint8_t* may, uint32_t* n_may, uint32_t mode,
          void* stream) {
  if (n == 0) return LSBM_OK;
  if (!base || !handles || !keys || !key_offsets || !may ||
      (mode == kProbeFilterBlock && !data_offsets))
    return engine_fail(LSBM_ERR_INVALID, "null pointer");
  if (bits_per_key < 0) return engine_fail(LSBM_ERR_INVALID, "bits_per_key < 0");
  int cus = 0;
  const int rc = engine_current_cus(&cus);
  if (rc != LSBM_OK) return rc;
  BloomProbeArgs a = {};
  a.base = base;
  a.handles = handles;
  a.data_offsets = data_offsets;
  a.keys = static_cast<const uint8_t*>(keys);
  a.key_offsets = key_offsets;
  a.may = may;
  a.n_may = n_may;
  a.n = n;
  a.k_use = lsbm_bloom_k_probe(bits_per_key, bloom_bits_use);
  a.strip = strip;
  a.mode = mode;
  // grid-stride: no more workgroups than are resident at once
  const hipError_t e = launch_bloom_probe(a, grid_for(cus, n, 256, bloom_probe_blocks_per_cu(mode)),
                                          static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : engine_fail_hip(e, "bloom_probe_kernel");
}

}  // namespace
}  // namespace lsbm

using namespace lsbm;

extern "C" {

__attribute__((visibility("default"))) int lsbm_bloom_build_dev(
    const void* d_keys, const uint64_t* d_key_offsets, uint32_t strip,
    const uint64_t* d_filter_first, const uint64_t* d_filter_out, uint64_t n_filters,
    int bits_per_key, uint8_t* d_out, void* stream) {
  if (n_filters == 0) return LSBM_OK;
  if (!d_keys || !d_key_offsets || !d_filter_first || !d_filter_out || !d_out)
    return engine_fail(LSBM_ERR_INVALID, "null pointer");
  if (bits_per_key < 0) return engine_fail(LSBM_ERR_INVALID, "bits_per_key < 0");
  int cus = 0;
  const int rc = engine_current_cus(&cus);
  if (rc != LSBM_OK) return rc;
  BloomBuildArgs a = {};
  a.keys = static_cast<const uint8_t*>(d_keys);
  a.key_offsets = d_key_offsets;
  a.filter_first = d_filter_first;
  a.filter_out = d_filter_out;
  a.out = d_out;
  a.n_filters = n_filters;
  a.bits_per_key = (uint64_t)bits_per_key;
  a.strip = strip;
  a.k = lsbm_bloom_k(bits_per_key);
  // one wave per range of filters (groups of kBloomGroup); no more
  // workgroups than are resident at once
  const uint64_t groups = (n_filters + kBloomGroup - 1) / kBloomGroup;
  const hipError_t e = launch_bloom_build(a, grid_for(cus, groups, kBloomWaves, bloom_build_blocks_per_cu()),
                                          static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : engine_fail_hip(e, "bloom_build_kernel");
}

__attribute__((visibility("default"))) int lsbm_bloom_may_match_dev(
    const uint8_t* d_filters, const uint64_t* d_filter_handles, const void* d_keys,
    const uint64_t* d_key_offsets, uint32_t strip, uint64_t n_queries, int bits_per_key,
    int bloom_bits_use, uint8_t* d_may, uint32_t* d_n_may, void* stream) {
  return probe(d_filters, d_filter_handles, nullptr, d_keys, d_key_offsets, strip, n_queries,
               bits_per_key, bloom_bits_use, d_may, d_n_may, kProbeFilter, stream);
}

__attribute__((visibility("default"))) int lsbm_filter_block_may_match_dev(
    const uint8_t* d_blocks, const uint64_t* d_block_handles, const uint64_t* d_data_offsets,
    const void* d_keys, const uint64_t* d_key_offsets, uint32_t strip, uint64_t n_queries,
    int bits_per_key, int bloom_bits_use, uint8_t* d_may, uint32_t* d_n_may, void* stream) {
  return probe(d_blocks, d_block_handles, d_data_offsets, d_keys, d_key_offsets, strip,
               n_queries, bits_per_key, bloom_bits_use, d_may, d_n_may, kProbeFilterBlock,
               stream);
}

}  // extern "C"
