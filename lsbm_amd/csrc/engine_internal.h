// engine_internal.h -- what the bloom entry points (bloom_engine.cc) share
// with the CRC engine (crc32c_engine.cc): the per-thread error text behind
// lsbm_crc32c_last_error() and the per-device initialisation (one
// std::call_once per device; LSBM_ERR_NO_DEVICE without a usable device).
// Hidden symbols: not part of the C ABI.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace lsbm {

int engine_fail(int code, const char* what);            // records `what`, returns code
int engine_fail_hip(hipError_t e, const char* what);    // LSBM_ERR_HIP
int engine_current_cus(int* cus);  // initialises the current device; its CU count
// lsbm_sst_seal_dev in one pass, the trailers stored in place as plain byte
// stores (never the compare-and-swap merge): for an image the kernel reads
// and writes over PCIe (table_checksum.cc's zero copy), where device atomics
// on host memory are not to be relied on.
int sst_seal_in_place(uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles, const uint8_t* d_types,
                      uint64_t n_blocks, hipStream_t stream);

}  // namespace lsbm
