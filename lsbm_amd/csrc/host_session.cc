// host_session.cc -- see host_session.h.
#include "host_session.h"

#include <atomic>
#include <chrono>

#include <emmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsbm_crc32c.h"

namespace lsbm {

Status hip_status(hipError_t e, const char* what) {
  return Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

namespace {
bool pinned_byte(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" for pageable memory
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}
}  // namespace

// [p, p + n) page-locked: its first and last bytes are, and the allocation
// holding p (when the runtime reports one) spans the whole range, so that a
// registered prefix of a larger buffer does not pass as pinned.
bool host_pinned(const void* p, size_t n) {
  if (!p || n == 0 || !pinned_byte(p)) return false;
  const char* last = static_cast<const char*>(p) + (n - 1);
  if (!pinned_byte(last)) return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) == hipSuccess && base) {
    const char* b = static_cast<const char*>(base);
    return static_cast<const char*>(p) >= b && last < b + size;
  }
  (void)hipGetLastError();
  return true;
}

// ---- worker pool: one job at a time, the caller works on it too ----
namespace {

// set on the pool's threads, and on a caller while it works on its own job
thread_local bool t_in_pool = false;

class WorkPool {
 public:
  void run(size_t pieces, const std::function<void(size_t)>& fn) {
    std::lock_guard<std::mutex> job(job_mu_);
    start();
    {
      std::lock_guard<std::mutex> l(mu_);
      fn_ = &fn;
      pieces_ = pieces;
      next_ = finished_ = 0;
      gen_++;
    }
    cv_.notify_all();
    t_in_pool = true;
    work();
    t_in_pool = false;
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return finished_ == pieces_; });
    fn_ = nullptr;
  }

 private:
  void start() {
    if (!threads_.empty()) return;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    // (the caller is the 16th: the one-GPU box's CPU share is 16)
    const unsigned nt = std::min(15u, hw > 1 ? hw - 1 : 1u);
    for (unsigned t = 0; t < nt; t++)
      threads_.emplace_back([this] {
        t_in_pool = true;
        uint64_t seen = 0;
        for (;;) {
          {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return gen_ != seen; });
            seen = gen_;
          }
          work();
        }
      });
    for (auto& t : threads_) t.detach();  // parked on cv_ for the life of the process
  }
  void work() {
    for (;;) {
      size_t k;
      const std::function<void(size_t)>* fn;
      {
        std::lock_guard<std::mutex> l(mu_);
        if (next_ >= pieces_) return;
        k = next_++;
        fn = fn_;
      }
      (*fn)(k);
      std::lock_guard<std::mutex> l(mu_);
      if (++finished_ == pieces_) done_cv_.notify_all();
    }
  }
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> threads_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t pieces_ = 0, next_ = 0, finished_ = 0;
  uint64_t gen_ = 0;
};

WorkPool* pool() {
  static WorkPool* p = new WorkPool;  // never destroyed: its threads outlive static teardown
  return p;
}

constexpr int kMaxDevices = 64;
std::mutex g_reg;
HostSession* g_sessions[kMaxDevices] = {};

}  // namespace

void parallel_for(size_t pieces, const std::function<void(size_t)>& fn) {
  if (pieces == 1 || (pieces > 1 && t_in_pool)) {  // (nested: inline, the pool runs one job at a time)
    for (size_t k = 0; k < pieces; k++) fn(k);
    return;
  }
  if (pieces > 1) pool()->run(pieces, fn);
}

// memcpy into a staging buffer with non-temporal stores: the pinned buffer is
// only read again by the DMA engine, so its lines need not be read into the
// cache first (a plain store to a line the cache does not hold reads it):
// 2 host memory passes per byte instead of 3.  The pageable layers are bound
// by this copy (profiles/r03/check1/host_timing.log: 38-43 GB/s with memcpy).
// LSBM_HOST_COPY=plain keeps memcpy (A/B).
namespace {
bool plain_copy() {
  static const bool plain = [] {
    const char* v = getenv("LSBM_HOST_COPY");
    return v && v[0] == 'p';
  }();
  return plain;
}

void stream_copy(char* d, const char* s, size_t n) {
  if (n < 256 || plain_copy()) {
    memcpy(d, s, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
  memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 48), e);
  }
  _mm_sfence();  // (the stores are visible before the DMA that follows is enqueued)
  memcpy(d + i, s + i, n - i);
}
}  // namespace

void parallel_copy(void* dst, const void* src, size_t n) {
  constexpr size_t kPiece = 1u << 20;
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  if (n < (4u << 20)) {
    stream_copy(d, s, n);
    return;
  }
  parallel_for((n + kPiece - 1) / kPiece, [&](size_t k) {
    const size_t off = k * kPiece;
    stream_copy(d + off, s + off, std::min(kPiece, n - off));
  });
}

// ---- buffers ----
hipError_t StagePair::reserve(size_t bytes) {
  if (bytes <= cap && !mapped) return hipSuccess;
  release();
  bytes = std::max<size_t>(bytes, 1u << 16);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d), bytes);
  mapped = false;
  if (e != hipSuccess) {
    release();
    return e;
  }
  cap = bytes;
  return hipSuccess;
}

hipError_t StagePair::reserve_mapped(size_t bytes) {
  if (bytes <= cap && mapped) return hipSuccess;
  release();
  bytes = std::max<size_t>(bytes, 1u << 16);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&h), bytes,
                               hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0);
  if (e != hipSuccess) {
    if (h) (void)hipHostFree(h);
    h = d = nullptr;
    return e;
  }
  mapped = true;
  cap = bytes;
  return hipSuccess;
}

void StagePair::release() {
  if (h) (void)hipHostFree(h);
  if (d && !mapped) (void)hipFree(d);
  h = d = nullptr;
  cap = 0;
  mapped = false;
}

// ---- session ----
hipError_t HostSession::init() {
  for (Stage& s : stage_) {
    hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

HostSession::~HostSession() {
  DeviceGuard g(device_);
  for (Stage& s : stage_) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.bulk.release();
    s.meta.release();
    s.res.release();
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  for (int k = 0; k < kScratch; k++)
    if (scratch_[k]) (void)hipFree(scratch_[k]);
}

hipError_t HostSession::scratch(int k, size_t bytes, void** p) {
  if (bytes > scratch_cap_[k]) {
    if (scratch_[k]) {
      (void)hipStreamSynchronize(stage_[0].stream);
      (void)hipFree(scratch_[k]);
      scratch_[k] = nullptr;
      scratch_cap_[k] = 0;
    }
    const size_t cap = std::max<size_t>(bytes, 1u << 12);
    const hipError_t e = hipMalloc(&scratch_[k], cap);
    if (e != hipSuccess) return e;
    scratch_cap_[k] = cap;
  }
  *p = scratch_[k];
  return hipSuccess;
}

hipError_t HostSession::wait(Stage& s) {
  if (!s.busy) return hipSuccess;
  s.busy = false;
  return hipEventSynchronize(s.done);
}

hipError_t HostSession::upload(void* d, const void* h, size_t n) {
  if (n == 0) return hipSuccess;
  Stage& s0 = stage_[0];
  if (host_pinned(h, n)) {
    hipError_t e = hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s0.stream);
    return e == hipSuccess ? hipStreamSynchronize(s0.stream) : e;
  }
  // through the stages' pinned buffers: stage i's copy overlaps stage i-1's
  // DMA (on the other stages' streams, so stage 0's queue is drained first)
  hipError_t e0 = hipStreamSynchronize(s0.stream);
  if (e0 != hipSuccess) return e0;
  int i = 0;
  for (size_t off = 0; off < n; off += kChunkBytes, i = (i + 1) % kStages) {
    const size_t k = std::min(kChunkBytes, n - off);
    Stage& s = stage_[i];
    hipError_t e = wait(s);
    if (e == hipSuccess) e = s.bulk.reserve(kChunkBytes);
    if (e != hipSuccess) return e;
    parallel_copy(s.bulk.h, static_cast<const char*>(h) + off, k);
    e = hipMemcpyAsync(static_cast<char*>(d) + off, s.bulk.h, k, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) return e;
    s.busy = true;
  }
  for (Stage& s : stage_) {
    const hipError_t e = wait(s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t HostSession::download(void* h, const void* d, size_t n) {
  if (n == 0) return hipSuccess;
  Stage& s0 = stage_[0];
  // (everything the caller enqueued on stage 0's stream comes first)
  if (host_pinned(h, n)) {
    hipError_t e = hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s0.stream);
    return e == hipSuccess ? hipStreamSynchronize(s0.stream) : e;
  }
  hipError_t e = hipStreamSynchronize(s0.stream);
  if (e != hipSuccess) return e;
  const size_t chunks = (n + kChunkBytes - 1) / kChunkBytes;
  auto issue = [&](size_t c) -> hipError_t {
    Stage& s = stage_[c % kStages];
    const size_t off = c * kChunkBytes, k = std::min(kChunkBytes, n - off);
    hipError_t ee = s.bulk.reserve(kChunkBytes);
    if (ee == hipSuccess)
      ee = hipMemcpyAsync(s.bulk.h, static_cast<const char*>(d) + off, k, hipMemcpyDeviceToHost,
                          s.stream);
    if (ee == hipSuccess) ee = hipEventRecord(s.done, s.stream);
    if (ee == hipSuccess) s.busy = true;
    return ee;
  };
  for (size_t c = 0; c < chunks && c < (size_t)kStages; c++)
    if ((e = issue(c)) != hipSuccess) return e;
  for (size_t c = 0; c < chunks; c++) {
    Stage& s = stage_[c % kStages];
    if ((e = wait(s)) != hipSuccess) return e;
    const size_t off = c * kChunkBytes, k = std::min(kChunkBytes, n - off);
    parallel_copy(static_cast<char*>(h) + off, s.bulk.h, k);
    if (c + kStages < chunks && (e = issue(c + kStages)) != hipSuccess) return e;
  }
  return hipSuccess;
}

void HostSession::ShutdownAll() {
  std::lock_guard<std::mutex> l(g_reg);
  for (int dev = 0; dev < kMaxDevices; dev++) {
    HostSession* s = g_sessions[dev];
    if (!s) continue;
    {
      std::lock_guard<std::mutex> sl(s->mu_);  // no lease may be open
    }
    delete s;
    g_sessions[dev] = nullptr;
  }
}

// ---- lease ----
// Every exit path of a layer (an error between enqueueing a chunk and
// collecting it included) ends here: the stages' work is waited for and their
// results dropped, so that no later call collects a stale chunk (its tag would
// index that call's plan) and no DMA from the caller's memory is still in
// flight when the layer returns.
SessionLease::~SessionLease() {
  if (s_)
    for (int i = 0; i < HostSession::kStages; i++) {
      Stage& sg = s_->stage(i);
      if (sg.stream) (void)hipStreamSynchronize(sg.stream);
      sg.busy = false;
    }
  if (lock_.owns_lock()) lock_.unlock();
  delete guard_;
}

namespace {
std::atomic<int> g_fault_after{-1};
bool timing_on() {
  static const bool on = [] {
    const char* v = getenv("LSBM_HOST_TIMING");
    return v && v[0] == '1';
  }();
  return on;
}
}  // namespace

double HostTiming::now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
HostTiming::HostTiming(const char* w) : what(w), on(timing_on()), t0(on ? now() : 0.0) {}
HostTiming::~HostTiming() {
  if (on)
    fprintf(stderr, "{\"host_timing\": \"%s\", \"total_ms\": %.3f, \"copy_ms\": %.3f, \"wait_ms\": %.3f, \"post_ms\": %.3f, "
            "\"prep_ms\": %.3f, \"enqueue_ms\": %.3f}\n",
            what, (now() - t0) * 1e3, t[kCopy] * 1e3, t[kWait] * 1e3, t[kPost] * 1e3, t[kPrep] * 1e3,
            t[kEnqueue] * 1e3);
}

bool host_fault_point(size_t enqueued) {
  int n = g_fault_after.load();
  if (n < 0 || enqueued < (size_t)n) return false;
  return g_fault_after.compare_exchange_strong(n, -1);
}

Status SessionLease::Open(int device) {
  if (device < 0 || device >= kMaxDevices) return Status::InvalidArgument("bad device ordinal");
  if (lsbm_crc32c_init(device) != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
  guard_ = new DeviceGuard(device);
  if (guard_->status() != hipSuccess) return hip_status(guard_->status(), "hipSetDevice");
  HostSession* s = nullptr;
  {
    std::lock_guard<std::mutex> l(g_reg);
    s = g_sessions[device];
    if (!s) {
      s = new HostSession(device);
      const hipError_t e = s->init();  // streams on `device` (current)
      if (e != hipSuccess) {
        delete s;
        return hip_status(e, "session streams");
      }
      g_sessions[device] = s;
    }
  }
  lock_ = std::unique_lock<std::mutex>(s->mu_);
  s_ = s;
  return Status::OK();
}

}  // namespace lsbm

// Testing only (include/lsbm_crc32c.h): the next host-layer pipeline fails
// once it has enqueued `chunks` chunks (-1: off).
extern "C" __attribute__((visibility("default"))) int lsbm_test_fail_host_pipeline(int chunks) {
  lsbm::g_fault_after.store(chunks < 0 ? -1 : chunks);
  return 0;
}
