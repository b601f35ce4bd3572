// host_stage.h -- host <-> device copies for the C++ host layers
// (table_checksum.cc, log_checksum.cc).
//
// Every copy goes through a page-locked bounce buffer with hipMemcpyAsync on
// the caller's stream.  A synchronous hipMemcpy from pageable memory into a
// buffer that reuses the address of a freed one was measured to leave the
// next kernel reading the OLD bytes on MI355X (ROCm 7.2; DESIGN.md section 5,
// "Staging"); the pinned async path is the one the engine's host-staged
// batches use and never showed it.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace lsbm {

class PinnedBounce {
 public:
  PinnedBounce() = default;
  ~PinnedBounce() {
    if (buf_) (void)hipHostFree(buf_);
  }
  PinnedBounce(const PinnedBounce&) = delete;
  PinnedBounce& operator=(const PinnedBounce&) = delete;

  hipError_t to_device(void* dst, const void* src, size_t n, hipStream_t s) {
    for (size_t off = 0; off < n;) {
      const size_t k = n - off < kChunk ? n - off : kChunk;
      hipError_t e = ensure();
      if (e == hipSuccess) e = hipStreamSynchronize(s);  // the bounce buffer is free again
      if (e != hipSuccess) return e;
      memcpy(buf_, static_cast<const char*>(src) + off, k);
      e = hipMemcpyAsync(static_cast<char*>(dst) + off, buf_, k, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return e;
      off += k;
    }
    return hipStreamSynchronize(s);
  }

  hipError_t to_host(void* dst, const void* src, size_t n, hipStream_t s) {
    for (size_t off = 0; off < n;) {
      const size_t k = n - off < kChunk ? n - off : kChunk;
      hipError_t e = ensure();
      if (e == hipSuccess)
        e = hipMemcpyAsync(buf_, static_cast<const char*>(src) + off, k, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) return e;
      memcpy(static_cast<char*>(dst) + off, buf_, k);
      off += k;
    }
    return hipSuccess;
  }

 private:
  static constexpr size_t kChunk = 8u << 20;
  hipError_t ensure() { return buf_ ? hipSuccess : hipHostMalloc(&buf_, kChunk, hipHostMallocDefault); }
  void* buf_ = nullptr;
};

// A non-blocking stream for one host-layer call.
class CallStream {
 public:
  CallStream() { err_ = hipStreamCreateWithFlags(&s_, hipStreamNonBlocking); }
  ~CallStream() {
    if (err_ == hipSuccess) (void)hipStreamDestroy(s_);
  }
  CallStream(const CallStream&) = delete;
  CallStream& operator=(const CallStream&) = delete;
  hipError_t status() const { return err_; }
  hipStream_t get() const { return s_; }

 private:
  hipStream_t s_ = nullptr;
  hipError_t err_;
};

}  // namespace lsbm
