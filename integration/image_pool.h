// integration/image_pool.h -- table images reused from table to table, and
// kept page-locked, for the GPU ends of lsbm's table code
// (integration/table_builder_gpu.cc's TableBuilder, gpu_table_reader.h's
// OpenVerifiedTable, GpuTableBuilder's image).
//
// Why: a fresh multi-MiB buffer per table is fresh memory each time -- every
// page faults in while the table is read or built, is page-locked by the GPU
// call for its duration, unlocked, and unmapped when the table is done.
// Measured on lsbm's db_bench (10M writes, 340 tables): +1.5-2 s of host CPU
// against the reference and its writer 20% slower, until the builder's images
// were pooled.  A pooled image keeps its pages, and
// (LSBM_TABLE_REGISTER, default on) stays page-locked at its current address
// and capacity through lsbm_host_register -- the library's own bookkeeping,
// so the registration never overlaps a page another thread's call has locked,
// and counts against LSBM_PINNED_MB -- and a seal or verify DMAs it in place
// with no per-call lock.  Before the string can move (a table that outgrows
// it), the registration is dropped (Moving) -- memory is never freed while
// registered.
//
// Header-only; links against liblsbm_crc32c.so (include/lsbm_crc32c.h).
#ifndef LSBM_INTEGRATION_IMAGE_POOL_H_
#define LSBM_INTEGRATION_IMAGE_POOL_H_

#include <stdlib.h>

#include <mutex>
#include <string>
#include <vector>

#include "lsbm_crc32c.h"

namespace leveldb {

struct PooledImage {
  std::string bytes;           // the image (its size is the caller's business)
  void* registered = nullptr;  // the range page-locked for it, if any
  size_t registered_bytes = 0;
};

class ImagePool {
 public:
  // the process's pool
  static ImagePool& Default() {
    static ImagePool* pool = new ImagePool();  // (kept until exit: teardown releases its buffers)
    return *pool;
  }

  // An image with capacity for `bytes` (grown here, unlocked first).
  PooledImage* Take(size_t bytes) {
    PooledImage* p = nullptr;
    {
      std::lock_guard<std::mutex> l(mu_);
      if (!free_.empty()) {
        p = free_.back();
        free_.pop_back();
      }
    }
    if (!p) p = new PooledImage();
    if (bytes > p->bytes.capacity()) {
      Moving(p);
      p->bytes.reserve(bytes);
    }
    return p;
  }

  // The image is about to move (a table outgrew it): unlock it first.  Also
  // the GpuTableBuilder image-move observer (arg: the PooledImage).
  static void Moving(void* arg) {
    PooledImage* p = static_cast<PooledImage*>(arg);
    if (p->registered) (void)lsbm_host_unregister(p->registered);
    p->registered = nullptr;
    p->registered_bytes = 0;
  }

  // Back into the pool, page-locked at its current address and capacity.
  void Give(PooledImage* p) {
    if (Register() && p->bytes.capacity() >= (1u << 20)) {
      void* at = &p->bytes[0];
      const size_t n = p->bytes.capacity();
      if (p->registered != at || p->registered_bytes != n) {
        Moving(p);
        // through the library, inside its page-lock bookkeeping: never over a
        // page another thread's image holds locked for a call, never a page
        // another image's in-place DMA relies on, and within LSBM_PINNED_MB
        // (refused: the image stays pooled, page-locked per call instead)
        if (lsbm_host_register(at, n) == 0) {
          p->registered = at;
          p->registered_bytes = n;
        }
      }
    }
    std::lock_guard<std::mutex> l(mu_);
    free_.push_back(p);
  }

  static bool Register() {
    static const bool on = [] {
      const char* e = getenv("LSBM_TABLE_REGISTER");
      return !(e && *e == '0');
    }();
    return on;
  }

 private:
  std::mutex mu_;
  std::vector<PooledImage*> free_;
};

}  // namespace leveldb

#endif  // LSBM_INTEGRATION_IMAGE_POOL_H_
