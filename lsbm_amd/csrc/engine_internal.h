// engine_internal.h -- what the bloom entry points (bloom_engine.cc) share
// with the CRC engine (crc32c_engine.cc): the per-thread error text behind
// lsbm_crc32c_last_error() and the per-device initialisation (one
// std::call_once per device; LSBM_ERR_NO_DEVICE without a usable device).
// Hidden symbols: not part of the C ABI.
#pragma once
#include <hip/hip_runtime_api.h>

namespace lsbm {

int engine_fail(int code, const char* what);            // records `what`, returns code
int engine_fail_hip(hipError_t e, const char* what);    // LSBM_ERR_HIP
int engine_current_cus(int* cus);  // initialises the current device; its CU count

}  // namespace lsbm
