// snappy_engine.cc -- the entry points of include/lsbm_snappy.h.
//
// Validates arguments, sizes the grid and launches snappy_kernels.hip on the
// caller's stream.  Never computes a batch on the CPU: without a usable device
// every entry point returns LSBM_ERR_NO_DEVICE.
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/lsbm_snappy.h"
#include "engine_internal.h"
#include "snappy_types.h"

namespace lsbm {

// launchers (snappy_kernels.hip)
hipError_t launch_snappy_length(const SnapLenArgs& a, int grid, hipStream_t stream);
hipError_t launch_snappy_uncompress(const SnapDecArgs& a, int grid, hipStream_t stream);
hipError_t launch_snappy_uncompress_deferred(const SnapDecArgs& a, int tier, int grid, hipStream_t stream);
hipError_t launch_snappy_compress(const SnapEncArgs& a, int grid, hipStream_t stream);
hipError_t launch_snappy_compress_mid(const SnapEncArgs& a, int grid, hipStream_t stream);
hipError_t launch_snappy_compress_large(const SnapEncArgs& a, int grid, hipStream_t stream);

namespace {

// one wave per block: at most as many single-wave workgroups as LDS keeps
// resident, grid-stride beyond that
int wave_grid(int cus, uint64_t n, uint32_t wgs_per_cu) {
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(n, (uint64_t)cus * wgs_per_cu));
}

}  // namespace
}  // namespace lsbm

using namespace lsbm;

extern "C" {

__attribute__((visibility("default"))) uint64_t lsbm_snappy_max_compressed_length(uint64_t n) {
  return 32 + n + n / 6;
}

__attribute__((visibility("default"))) int lsbm_snappy_compress_dev(
    const void* d_base, const uint64_t* d_offsets, uint64_t n, uint8_t* d_out,
    const uint64_t* d_out_offsets, uint64_t* d_out_len, void* stream) {
  if (n == 0) return LSBM_OK;
  if (!d_base || !d_offsets || !d_out || !d_out_offsets || !d_out_len)
    return engine_fail(LSBM_ERR_INVALID, "null pointer");
  int cus = 0;
  const int rc = engine_current_cus(&cus);
  if (rc != LSBM_OK) return rc;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SnapEncArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.out = d_out;
  a.out_offsets = d_out_offsets;
  a.out_len = d_out_len;
  a.n = n;
  // pass 1: one-fragment blocks that fit a 22 KiB LDS slice; the middle pass:
  // the ones it deferred (out_len = kSnapDeferred, scanned 64 per wave) that
  // fit 48 KiB; the last pass: the rest, the table in LDS, the bytes in global
  hipError_t e = launch_snappy_compress(a, wave_grid(cus, n, kSnapEncWgsPerCu), s);
  if (e != hipSuccess) return engine_fail_hip(e, "snappy_compress_kernel");
  e = launch_snappy_compress_mid(a, wave_grid(cus, (n + kSnapDecScan - 1) / kSnapDecScan, kSnapEncMidWgsPerCu), s);
  if (e != hipSuccess) return engine_fail_hip(e, "snappy_compress_mid_kernel");
  e = launch_snappy_compress_large(a, wave_grid(cus, (n + kSnapDecScan - 1) / kSnapDecScan, kSnapEncLargeWgsPerCu), s);
  return e == hipSuccess ? LSBM_OK : engine_fail_hip(e, "snappy_compress_large_kernel");
}

__attribute__((visibility("default"))) int lsbm_snappy_uncompressed_length_dev(
    const void* d_base, const uint64_t* d_offsets, uint64_t n, uint64_t* d_ulen, uint8_t* d_ok,
    void* stream) {
  if (n == 0) return LSBM_OK;
  if (!d_base || !d_offsets || !d_ulen || !d_ok) return engine_fail(LSBM_ERR_INVALID, "null pointer");
  int cus = 0;
  const int rc = engine_current_cus(&cus);
  if (rc != LSBM_OK) return rc;
  SnapLenArgs a = {static_cast<const uint8_t*>(d_base), d_offsets, d_ulen, d_ok, n};
  const uint64_t wgs = (n + 255) / 256;
  const int grid = (int)std::min<uint64_t>(wgs, (uint64_t)cus * 8);
  const hipError_t e = launch_snappy_length(a, grid, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : engine_fail_hip(e, "snappy_length_kernel");
}

__attribute__((visibility("default"))) int lsbm_snappy_uncompress_dev(
    const void* d_base, const uint64_t* d_offsets, uint64_t n, uint8_t* d_out,
    const uint64_t* d_out_offsets, uint8_t* d_ok, uint32_t* d_n_bad, void* stream) {
  if (n == 0) return LSBM_OK;
  if (!d_base || !d_offsets || !d_out || !d_out_offsets || !d_ok)
    return engine_fail(LSBM_ERR_INVALID, "null pointer");
  int cus = 0;
  const int rc = engine_current_cus(&cus);
  if (rc != LSBM_OK) return rc;
  SnapDecArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.out = d_out;
  a.out_offsets = d_out_offsets;
  a.ok = d_ok;
  a.n_bad = d_n_bad;
  a.n = n;
  // pass 1: blocks that fit a small LDS slice; passes 2-5: the ones the pass
  // before deferred (ok = 2 .. 5), scanned 16 per wave, in 9, 17, 33 and 80
  // KiB slices, the last one decoding what is left against global memory
  const hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = launch_snappy_uncompress(a, wave_grid(cus, n, kSnapDecWgsPerCu), s);
  if (e != hipSuccess) return engine_fail_hip(e, "snappy_uncompress_kernel");
  for (int t = 0; t < kSnapDecTiers; t++) {
    e = launch_snappy_uncompress_deferred(a, t, wave_grid(cus, (n + kSnapDecScan - 1) / kSnapDecScan,
                                                          (int)(160 * 1024 / kSnapDecTierLds[t])), s);
    if (e != hipSuccess) return engine_fail_hip(e, "snappy_uncompress_deferred_kernel");
  }
  return LSBM_OK;
}

}  // extern "C"
