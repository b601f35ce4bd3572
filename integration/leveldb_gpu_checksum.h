// integration/leveldb_gpu_checksum.h -- the Level-2 binding:
// what a maintainer adds to the reference's table/ to seal and verify the
// trailers of a whole table image held in device memory through the C ABI
// (include/lsbm_crc32c.h).  Written against the reference's own types
// (leveldb::BlockHandle, leveldb::Status, EncodeFixed32: table/format.h,
// include/leveldb/status.h, util/coding.h).  Compiled and linked with the
// reference's table/ and util/ objects by oracle/Makefile `gpubind`
// (tests/test_ref_link.py) and run on the GPU by tests/test_gpu_parity.py.
//
// Replaces, for a batch of blocks:
//   TableBuilder::WriteRawBlock's trailer (table/table_builder.cc:237-255)
//   ReadBlock's checksum check            (table/format.cc:95-103)
#ifndef LSBM_INTEGRATION_LEVELDB_GPU_CHECKSUM_H_
#define LSBM_INTEGRATION_LEVELDB_GPU_CHECKSUM_H_

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

#include "leveldb/status.h"
#include "lsbm_crc32c.h"
#include "table/format.h"
#include "util/coding.h"

namespace leveldb {

// WriteRawBlock for every block of a table image already in device memory
// (d_file, file_bytes): the trailers' crc fields come back densely (4 B per
// block, lsbm_sst_trailer_crcs_dev) and the host writes each trailer into its
// own copy of the file, exactly where WriteRawBlock appends it.
inline Status SealTrailersOnGpu(const uint8_t* d_file, uint64_t file_bytes, char* host_file,
                                const std::vector<BlockHandle>& h, const std::vector<uint8_t>& types,
                                hipStream_t s) {
  const size_t n = h.size();
  if (n == 0) return Status::OK();
  if (types.size() != n) return Status::InvalidArgument("gpu seal", "one type per block");
  std::vector<uint64_t> hh(2 * n);
  for (size_t i = 0; i < n; i++) {
    hh[2 * i] = h[i].offset();
    hh[2 * i + 1] = h[i].size();
  }
  uint64_t* d_h = nullptr;
  uint8_t* d_t = nullptr;
  uint32_t* d_m = nullptr;
  uint32_t* d_bad = nullptr;
  std::vector<uint32_t> m(n);
  uint32_t nbad = 0;
  // the first failing HIP call outside the library (its message, not the
  // library's last error, goes into the Status), or the library's return code
  hipError_t herr = hipSuccess;
  int rc = LSBM_OK;
  auto hip = [&](hipError_t e) {
    if (e != hipSuccess && herr == hipSuccess) herr = e;
    return herr == hipSuccess;
  };
  if (hip(hipMallocAsync(reinterpret_cast<void**>(&d_h), hh.size() * 8, s)) &&
      hip(hipMallocAsync(reinterpret_cast<void**>(&d_t), n, s)) &&
      hip(hipMallocAsync(reinterpret_cast<void**>(&d_m), n * 4, s)) &&
      hip(hipMallocAsync(reinterpret_cast<void**>(&d_bad), 4, s)) &&
      hip(hipMemcpyAsync(d_h, hh.data(), hh.size() * 8, hipMemcpyHostToDevice, s)) &&
      hip(hipMemcpyAsync(d_t, types.data(), n, hipMemcpyHostToDevice, s)) &&
      hip(hipMemsetAsync(d_bad, 0, 4, s))) {
    rc = lsbm_sst_trailer_crcs_dev(d_file, file_bytes, d_h, d_t, n, d_m, d_bad, s);
    if (rc == LSBM_OK) {
      (void)(hip(hipMemcpyAsync(m.data(), d_m, n * 4, hipMemcpyDeviceToHost, s)) &&
             hip(hipMemcpyAsync(&nbad, d_bad, 4, hipMemcpyDeviceToHost, s)));
    }
  }
  if (d_h) (void)hipFreeAsync(d_h, s);
  if (d_t) (void)hipFreeAsync(d_t, s);
  if (d_m) (void)hipFreeAsync(d_m, s);
  if (d_bad) (void)hipFreeAsync(d_bad, s);
  (void)hip(hipStreamSynchronize(s));
  if (rc != LSBM_OK) return Status::IOError("gpu seal", lsbm_crc32c_last_error());
  if (herr != hipSuccess) return Status::IOError("gpu seal", hipGetErrorString(herr));
  if (nbad) return Status::Corruption("truncated block read");  // a handle past the image
  for (size_t i = 0; i < n; i++) {  // table/table_builder.cc:245-249
    char* t = host_file + h[i].offset() + h[i].size();
    t[0] = static_cast<char>(types[i]);
    EncodeFixed32(t + 1, m[i]);
  }
  return Status::OK();
}

// ReadBlock's checksum check for n blocks of a device-resident image (handles
// as {offset, size} pairs in device memory): ok[i] per block, and the status
// ReadBlock would return for the first bad one -- Corruption("truncated block
// read") for a handle whose n + 5 bytes leave the image (table/format.cc:88-91),
// else Corruption("block checksum mismatch") (:95-103).  Only when some block
// fails are ok[] and the handles copied back, to find that first one.
inline Status VerifyBlocksOnGpu(const uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles,
                                uint64_t n, uint8_t* d_ok, uint32_t* d_nbad, hipStream_t s) {
  hipError_t e = hipMemsetAsync(d_nbad, 0, 4, s);
  if (e != hipSuccess) return Status::IOError("gpu verify", hipGetErrorString(e));
  if (lsbm_sst_verify_dev(d_file, file_bytes, d_handles, n, d_ok, d_nbad, s) != LSBM_OK)
    return Status::IOError("gpu verify", lsbm_crc32c_last_error());
  uint32_t nbad = 0;
  e = hipMemcpyAsync(&nbad, d_nbad, 4, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return Status::IOError("gpu verify", hipGetErrorString(e));
  if (nbad == 0) return Status::OK();
  std::vector<uint8_t> ok(n);
  std::vector<uint64_t> hh(2 * n);
  e = hipMemcpyAsync(ok.data(), d_ok, n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(hh.data(), d_handles, 2 * n * 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return Status::IOError("gpu verify", hipGetErrorString(e));
  for (uint64_t i = 0; i < n; i++) {
    if (ok[i]) continue;
    const uint64_t off = hh[2 * i], size = hh[2 * i + 1];
    const bool truncated = off > file_bytes || size > file_bytes - off ||
                           file_bytes - off - size < kBlockTrailerSize;
    return Status::Corruption(truncated ? "truncated block read" : "block checksum mismatch");
  }
  return Status::Corruption("block checksum mismatch");
}

}  // namespace leveldb

#endif  // LSBM_INTEGRATION_LEVELDB_GPU_CHECKSUM_H_
