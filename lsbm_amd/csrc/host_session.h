// host_session.h -- persistent per-device staging for the C++ host layers
// (table_checksum.cc, log_checksum.cc, filter_block.cc, block_compression.cc)
// and the host-staged batch entry point (crc32c_engine.cc).
//
// A HostSession belongs to one device and is created on that device when a
// layer needs one and none is idle (up to LSBM_HOST_SESSIONS, default 8, per
// device: concurrent callers on one device each lease their own): kStages
// pipeline stages, each a non-blocking
// stream, a completion event and three pinned-host / device buffer pairs
// (bulk bytes, per-item inputs, per-item results) that grow on demand and are
// kept, plus a few device scratch buffers for single-shot layers.  Nothing is
// allocated per call once the buffers have reached their working size;
// lsbm_crc32c_shutdown() frees everything.
//
// Copies into pinned memory are the host's share of the work: copies of 4 MiB
// and more are split over a pool of worker threads so that the staging
// keeps up with PCIe (~55 GB/s measured for pinned H2D on the MI355X box).
// The pinned buffers sit on the device's NUMA node (host_numa.h), and the
// session's copy jobs go to that node's workers first.
// A source that is already page-locked (hipHostMalloc / hipHostRegister) is
// DMA-ed directly.  All DMA is stream-ordered hipMemcpyAsync on the stage's
// stream: a synchronous hipMemcpy from pageable memory may return before its
// DMA has landed and is not ordered with a non-blocking stream (the stale-
// bytes race DESIGN.md section 5 records).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <mutex>

#include "../../include/lsbm/status.h"

namespace lsbm {

// Makes `device` current for a scope and restores the caller's device after.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    have_prev_ = hipGetDevice(&prev_) == hipSuccess;
    err_ = hipSetDevice(device);
  }
  ~DeviceGuard() {
    if (have_prev_) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
  hipError_t status() const { return err_; }

 private:
  int prev_ = 0;
  bool have_prev_ = false;
  hipError_t err_;
};

// A pinned host buffer and a device buffer of the same capacity.  A *mapped*
// pair (reserve_mapped) is one coherent page-locked host buffer that `d`
// addresses from the device: a kernel's results land in host memory with no
// copy.  The layers take their per-block results this way: a device-to-host
// copy queued behind the next chunk's bulk host-to-device copy finished
// ~0.6 ms after its kernel and held the stage (profiles/r03/host_trace).
struct StagePair {
  uint8_t* h = nullptr;
  uint8_t* d = nullptr;
  size_t cap = 0;
  bool mapped = false;
  int node = -1;    // NUMA node of the host pages (-1: HIP's default placement)
  int device = -1;  // the session's device (pinned-bytes accounting)
  hipError_t reserve(size_t bytes);  // grows (never shrinks); contents are not kept
  hipError_t reserve_mapped(size_t bytes);
  void release();

 private:
  hipError_t alloc(size_t bytes, bool map);
};

// One pipeline stage.
struct Stage {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  hipEvent_t copied = nullptr;  // this stage's DMA on the session's copy stream has landed
  bool busy = false;  // work enqueued whose results the caller has not collected
  // Within a lease: true only while the stream is known to be idle (the last
  // thing on it was an event that wait() has seen complete).  A layer clears
  // it before it enqueues; the lease's release then skips the stream sync of a
  // settled stage (an idle-stream hipStreamSynchronize is a GPU round trip,
  // 15-20 us, profiles/r04/one_table_trace/summary_call40.txt).
  bool settled = false;
  uint64_t tag = 0;   // the caller's chunk number
  double wait_ewma_us = 0;  // moving average of this stage's waits (HostSession::wait)
  StagePair bulk, meta, res;
  StagePair zmeta;  // mapped: per-block inputs the kernel reads in place (zero-copy table jobs)
};

class HostSession {
 public:
#ifndef LSBM_HOST_STAGES  // (A/B builds override)
#define LSBM_HOST_STAGES 4
#endif
#ifndef LSBM_HOST_CHUNK_MB
#define LSBM_HOST_CHUNK_MB 64
#endif
  static constexpr int kStages = LSBM_HOST_STAGES;
  static constexpr size_t kChunkBytes = (size_t)LSBM_HOST_CHUNK_MB << 20;  // bulk bytes per stage and chunk (at most)
  static constexpr size_t kMinChunkBytes = 2u << 20;
  // Chunk size for a job of `total` bytes: about a quarter of it, so that even
  // one table's copy, DMA and kernel overlap, within [2 MiB, 64 MiB].
  static size_t chunk_for(size_t total) {
    const size_t q = total / 4;
    return q < kMinChunkBytes ? kMinChunkBytes : (q > kChunkBytes ? kChunkBytes : q);
  }
  static constexpr int kScratch = 8;

  Stage& stage(int i) { return stage_[i]; }
  // Device scratch buffer k (k < kScratch), at least `bytes` long.
  hipError_t scratch(int k, size_t bytes, void** p);
  // Stage 0's stream, for a layer's own enqueues (so no longer settled).
  hipStream_t stream() {
    stage_[0].settled = false;
    return stage_[0].stream;
  }
  int device() const { return device_; }
  int node() const { return node_; }

  // Host -> device / device -> host of n bytes on stage 0's stream, through
  // the stages' pinned buffers (overlapped) unless `h` is page-locked.
  // Synchronous: returns when the bytes have arrived.
  hipError_t upload(void* d, const void* h, size_t n);
  hipError_t download(void* h, const void* d, size_t n);
  // upload of several host pieces laid back to back at d (a gather): the
  // stages' chunks are filled from as many pieces as they span, one DMA per
  // chunk, instead of one synchronous upload per piece.
  struct Piece {
    const void* h;
    size_t n;
  };
  hipError_t upload_pieces(void* d, const Piece* pieces, size_t count);

  // Waits for a stage's enqueued work (no-op if idle); clears busy.  Sleeps
  // in short naps while the work is expected to take longer than ~60 us more
  // (a moving average of the stage's waits), then spins (LSBM_WAIT=spin: spin
  // throughout).
  hipError_t wait(Stage& s);

  // The session's copy stream (created on first use): page-locked chunks'
  // DMAs all go through it, so they land one after another at the full link
  // rate and chunk c's kernel (on its stage's stream, after the stage's
  // `copied` event) runs under chunk c+1's DMA.  On four stage streams the
  // four DMAs of a table ran side by side and all landed at the end.
  hipError_t copy_stream(hipStream_t* out);

  // Frees every session (lsbm_crc32c_shutdown).
  static void ShutdownAll();
  // Frees this (idle) session's staging buffers; they grow again on demand.
  void release_staging();

 private:
  friend class SessionLease;
  explicit HostSession(int device) : device_(device) {}
  ~HostSession();
  hipError_t init();
  int device_;
  int node_ = -1;
  Stage stage_[kStages];
  hipStream_t copy_stream_ = nullptr;
  bool copy_pending_ = false;  // copies enqueued during the current lease
  void* scratch_[kScratch] = {};
  size_t scratch_cap_[kScratch] = {};
};

// One of the device's sessions, held by this caller alone, with the device
// current for the lease's lifetime (the caller's current device is restored
// after) and the caller's pool jobs steered to the device's NUMA node.  On
// release every stage is drained and marked idle, whatever the caller left,
// and the session goes back to the device's idle list.
class SessionLease {
 public:
  SessionLease() = default;
  ~SessionLease();
  SessionLease(const SessionLease&) = delete;
  SessionLease& operator=(const SessionLease&) = delete;
  // Initialises the device (lsbm_crc32c_init) and its session.
  Status Open(int device);
  HostSession* operator->() const { return s_; }
  HostSession& operator*() const { return *s_; }

 private:
  HostSession* s_ = nullptr;
  DeviceGuard* guard_ = nullptr;
  int prev_node_ = -1;
  bool node_set_ = false;  // Open got as far as steering this thread's jobs
};

// Sessions created so far for `device` (idle or leased), and the page-locked
// staging bytes they hold (kept under LSBM_PINNED_MB per device, default
// 1024, by trimming idle sessions when a lease is released).
int session_count(int device);
size_t pinned_bytes(int device);

// Is [p, p + n) inside page-locked host memory (hipHostMalloc'd or registered)
// that stays locked for the caller's call?  Not if a page of it is held by
// another call's CallLocks (that call unlocks it when it returns).
bool host_pinned(const void* p, size_t n);
// Long-lived registrations (lsbm_host_register / lsbm_host_unregister, the C
// ABI's): 0 or -1, and the bytes registered so far.
int host_register(const void* p, size_t n);
int host_unregister(const void* p);
size_t host_registered_bytes();

// Page-locks a call's pageable images (hipHostRegister: ~1 us, the pages are
// pinned by the DMA that reads them) so that they are DMA-ed in place with no
// staging copy, and unlocks them when destroyed.  Declare it BEFORE the
// call's SessionLease: the lease, destroyed first, has synchronised every
// stream that may still read an image.  The device only reads the images
// (hipHostRegisterReadOnly where the device supports it, so read-only
// mappings such as an mmap'd table file qualify; else only images the caller
// passed as writable).  LSBM_AUTO_LOCK=0 turns it off (staging copies).
// Thread-safe: registrations and unregistrations of all calls are serialised
// under one process-wide mutex, and a range that shares a page with another
// live call's lock is neither locked nor taken as page-locked (host_pinned):
// concurrent callers whose images are neighbours on the heap stage instead.
class CallLocks {
 public:
  CallLocks() = default;
  CallLocks(const CallLocks&) = delete;
  CallLocks& operator=(const CallLocks&) = delete;
  ~CallLocks();
  // true when [p, p + n) is page-locked for this call from here on (false: it
  // could not be, e.g. a page of it is registered already or held by another
  // call's lock; nothing changed)
  bool add(int device, const void* p, size_t n, bool writable);
  static bool enabled();

 private:
  struct Reg {
    void* p;
    uintptr_t lo;  // its first page (the key of its range in the lock set)
  };
  std::vector<Reg> regs_;
};

// Page ranges held by live CallLocks, and ranges locked since start-up (testing).
int locked_ranges();
long locks_taken();

// fn(0) ... fn(pieces - 1) over the worker pool and the caller; returns when
// all have run.  The pool has usable_cores() - 1 threads (the affinity mask
// capped by the cgroup CPU quota), grouped by NUMA node; jobs of concurrent
// callers run at the same time, each worker preferring jobs of its own node
// (the caller's session's device node).  At most max_helpers workers join
// the caller (-1: any; 0: the caller alone).  A call from inside a pool task
// runs its pieces inline on that thread (no deadlock, no extra parallelism).
// Idle workers spin at most LSBM_POOL_SPIN_US (20 us) and then sleep.
void parallel_for(size_t pieces, const std::function<void(size_t)>& fn, int max_helpers = -1);

// The pool's worker count (starts it), and, for tests, the most jobs that
// had pieces running at the same moment since the previous call.
int pool_threads();
int pool_take_peak_jobs();

// Workers that join a staging copy (LSBM_COPY_THREADS - 1; default 3).
int copy_helpers();

// memcpy of n bytes into pinned staging (non-temporal stores), split over the
// caller and copy_helpers() workers when n >= 256 KiB.
void parallel_copy(void* dst, const void* src, size_t n);

// Diagnostics (LSBM_HOST_TIMING=1 in the environment): a layer's pipeline
// adds the wall time of its phases and prints one line to stderr per call:
// the host copy into pinned staging, waits for a stage, the host-side result
// handling, per-chunk metadata, the enqueue calls, and the whole call.
struct HostTiming {
  enum Phase { kCopy, kWait, kPost, kPrep, kEnqueue, kPhases };
  explicit HostTiming(const char* what);
  ~HostTiming();
  void add(Phase p, double s) { t[p] += s; }
  static double now();
  const char* what;
  bool on;
  double t0, t[kPhases] = {0, 0, 0, 0, 0};
};

// Fault injection for the error-path tests (lsbm_test_fail_host_pipeline):
// true once, when a pipeline that has enqueued `enqueued` chunks reaches the
// armed count.
bool host_fault_point(size_t enqueued);

// Stage waits sleep on blocking-sync events instead of spinning
// (LSBM_BLOCKING_WAIT=1).
bool blocking_wait();

// Status for a failed HIP call.
Status hip_status(hipError_t e, const char* what);

}  // namespace lsbm
