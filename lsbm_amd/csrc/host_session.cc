// host_session.cc -- see host_session.h.
#include "host_session.h"

#include <atomic>
#include <chrono>

#include <emmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsbm_crc32c.h"
#include "host_numa.h"

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
static bool pinned_range(const void* p, size_t n) {
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
  // hipHostRegister'd memory reports no address range: the first and last
  // bytes must then belong to the same registration (one buffer id), so that
  // two registrations with an unregistered gap between them do not pass.
  // Unconfirmed: take the staging copy.
  unsigned long long id0 = 0, id1 = 0;
  if (hipPointerGetAttribute(&id0, HIP_POINTER_ATTRIBUTE_BUFFER_ID, const_cast<void*>(p)) == hipSuccess &&
      hipPointerGetAttribute(&id1, HIP_POINTER_ATTRIBUTE_BUFFER_ID, const_cast<char*>(last)) == hipSuccess)
    return id0 != 0 && id0 == id1;
  (void)hipGetLastError();
  return false;
}

// ---- the library's own per-call page locks ----
// Every page range the library locks for a call (CallLocks) is reserved, and
// every "is this range page-locked?" question the layers ask is answered,
// under one process-wide mutex, against the set of page ranges that live
// CallLocks hold (the registration itself runs outside it, on the reserved
// range, see CallLocks::add).  Round 4 checked "both ends unregistered" and
// then registered as two steps: two concurrent calls whose images share a
// page could both pass the check, and the loser's unregister could break the
// winner's registration with its DMA in flight.  Now:
//   * a range that touches a page a live CallLocks holds is never registered
//     again (it takes the staging copy);
//   * a range on such a page never counts as page-locked either: its bytes
//     may lie inside another call's registration, which that call drops when
//     it returns, so an in-place DMA from them could outlive it.
size_t host_register_budget();  // (LSBM_PINNED_MB, below)

namespace {
std::mutex g_lock_mu;
std::map<uintptr_t, uintptr_t> g_locked;  // [first page, end page) of each live CallLocks range
std::atomic<long> g_locks_taken{0};        // (testing: ranges locked since start-up)

// (the granularity of a registration: the system page)
uintptr_t page_size() {
  static const uintptr_t ps = [] {
    const long v = sysconf(_SC_PAGESIZE);
    return v > 0 ? (uintptr_t)v : (uintptr_t)4096;
  }();
  return ps;
}
uintptr_t page_lo(const void* p) { return reinterpret_cast<uintptr_t>(p) & ~(page_size() - 1); }
uintptr_t page_hi(const void* p, size_t n) {
  return (reinterpret_cast<uintptr_t>(p) + n + page_size() - 1) & ~(page_size() - 1);
}
// Long-lived registrations made through lsbm_host_register (an embedder's
// buffer pool, integration/image_pool.h): [first page, end page) -> the
// registered bytes.  Their pages are reserved like a CallLocks range's: no
// call registers over them, and no OTHER range on one of their pages counts
// as page-locked (its owner may unregister them at any time); a range inside
// the registered bytes does.
struct Persist {
  uintptr_t hi;
  const char* p;
  size_t n;
};
std::map<uintptr_t, Persist> g_persist;
size_t g_persist_bytes = 0;

// (under g_lock_mu)
bool touches_calls(uintptr_t lo, uintptr_t hi) {
  auto it = g_locked.lower_bound(hi);  // the first range starting at or after hi
  if (it == g_locked.begin()) return false;
  --it;
  return it->second > lo;
}
// the persistent registration whose pages [lo, hi) touches (nullptr: none);
// *more: it touches more than one
const Persist* touches_persist(uintptr_t lo, uintptr_t hi, bool* more) {
  *more = false;
  auto it = g_persist.lower_bound(hi);
  const Persist* hit = nullptr;
  while (it != g_persist.begin()) {
    --it;
    if (it->second.hi <= lo) break;
    if (hit) *more = true;
    hit = &it->second;
  }
  return hit;
}
bool touches_locked(uintptr_t lo, uintptr_t hi) {
  bool more;
  return touches_calls(lo, hi) || touches_persist(lo, hi, &more) != nullptr;
}
}  // namespace

bool host_pinned(const void* p, size_t n) {
  if (!p || n == 0) return false;
  std::lock_guard<std::mutex> l(g_lock_mu);
  const uintptr_t lo = page_lo(p), hi = page_hi(p, n);
  if (touches_calls(lo, hi)) return false;
  bool more = false;
  const Persist* r = touches_persist(lo, hi, &more);
  if (r) {  // only bytes inside one registration's own bytes
    const char* c = static_cast<const char*>(p);
    if (more || c < r->p || c + n > r->p + r->n) return false;
  }
  return pinned_range(p, n);
}

// lsbm_host_register: see include/lsbm_crc32c.h.
int host_register(const void* p, size_t n) {
  if (!p || n == 0) return -1;
  const uintptr_t lo = page_lo(p), hi = page_hi(p, n);
  {
    std::lock_guard<std::mutex> l(g_lock_mu);
    if (touches_locked(lo, hi)) return -1;  // (a live call's or another registration's pages)
    if (g_persist_bytes + n > host_register_budget()) return -1;
    hipPointerAttribute_t a;
    const char* c = static_cast<const char*>(p);
    for (const char* x : {c, c + n - 1}) {  // (never over an older registration)
      const hipError_t e = hipPointerGetAttributes(&a, x);
      (void)hipGetLastError();
      if (e == hipSuccess && a.type != hipMemoryTypeUnregistered) return -1;
    }
    g_persist.emplace(lo, Persist{hi, c, n});  // reserved
    g_persist_bytes += n;
  }
  if (hipHostRegister(const_cast<void*>(p), n, hipHostRegisterDefault) == hipSuccess) return 0;
  (void)hipGetLastError();
  std::lock_guard<std::mutex> l(g_lock_mu);
  g_persist.erase(lo);
  g_persist_bytes -= n;
  return -1;
}

int host_unregister(const void* p) {
  if (!p) return -1;
  uintptr_t lo;
  size_t n;
  {
    std::lock_guard<std::mutex> l(g_lock_mu);
    auto it = g_persist.find(page_lo(p));
    if (it == g_persist.end() || it->second.p != p) return -1;
    lo = it->first;
    n = it->second.n;
  }
  // unlocked first, then the reservation released (as ~CallLocks)
  const hipError_t e = hipHostUnregister(const_cast<void*>(p));
  (void)hipGetLastError();
  std::lock_guard<std::mutex> l(g_lock_mu);
  g_persist.erase(lo);
  g_persist_bytes -= n;
  return e == hipSuccess ? 0 : -1;
}

size_t host_registered_bytes() {
  std::lock_guard<std::mutex> l(g_lock_mu);
  return g_persist_bytes;
}

int locked_ranges() {
  std::lock_guard<std::mutex> l(g_lock_mu);
  return (int)g_locked.size();
}

long locks_taken() { return g_locks_taken.load(); }

// ---- worker pool: concurrent jobs, one thread group per NUMA node ----
//
// Each job is a piece counter over fn(0) .. fn(pieces - 1), with a cap on the
// pool workers that may join the caller on it (max_helpers).  Jobs from
// different callers (host layers on different devices, or several sessions
// of one device) run at the same time: a worker takes the next piece of the
// oldest job of its own node, else of the oldest job of any node, and the
// caller works on its own job too.  Sized from the CPUs the process may
// really use (usable_cores(): affinity mask capped by the cgroup quota),
// split over the nodes in proportion to their CPUs, each worker bound to its
// node's CPUs when there are several.
//
// CPU budget (round 5): a worker that finds nothing to take -- no job, or
// only jobs whose pieces are all claimed or whose helper cap is reached --
// spins at most spin_us() for the next publication, then sleeps until one.
// A publication wakes at most as many sleepers as the job can use.  Round 4's
// workers spun for as long as any job was published (every pool thread busy
// for a whole staged call: ~5 ms of CPU per 16 MiB table).
namespace {

// set on the pool's threads, and on a caller while it works on its own job
thread_local bool t_in_pool = false;
// the node whose workers a caller's jobs go to first (its session's device)
thread_local int t_job_node = -1;

struct Job {
  const std::function<void(size_t)>* fn;
  size_t pieces;
  int node;
  int max_helpers;
  // (each counter on a cache line of its own: every thread of the job hits
  // next once per piece, finished once per piece, and the caller polls it)
  alignas(64) std::atomic<size_t> next{0};
  alignas(64) std::atomic<size_t> finished{0};
  alignas(64) std::atomic<int> helpers{0};  // workers that joined (at most max_helpers)
  std::atomic<int> active{0};               // pieces in progress (testing: pool_take_peak_jobs)
};

// No lock on the way to a piece.  A job is published in a slot; a worker
// takes it with a hazard pointer (its own slot says "I may touch this job",
// then it re-reads the job slot), joins it if the helper cap allows, claims
// pieces with fetch_add and counts them done with another; the caller
// unpublishes its job, then waits until every piece is done and no worker's
// hazard names the job.  (The hazard is stored before the job slot is
// re-read, the job slot cleared before the hazards are read, all sequentially
// consistent: either the worker sees its job gone, or the caller sees the
// worker's hazard.)  The mutex is only for sleeping: a publication bumps gen_
// and then reads sleepers_; a worker about to sleep counts itself in
// sleepers_ and then re-reads gen_ (sequentially consistent, so one of the
// two sees the other: no lost wake-up).
// Round 4: with a mutex round trip per piece a parallel_for cost ~50 us; with
// one per worker and job (pick and drop), 25-37 us of empty pieces on 16
// threads (round 4; docs/DESIGN_HISTORY.md section 6).
class WorkPool {
 public:
  static constexpr int kJobSlots = 64;
  static constexpr int kMaxWorkers = 512;

  void run(size_t pieces, const std::function<void(size_t)>& fn, int node, int max_helpers) {
    start();
    Job j;
    j.fn = &fn;
    j.pieces = pieces;
    j.node = node;
    j.max_helpers = max_helpers < 0 ? kMaxWorkers : max_helpers;
    int slot = -1;
    if (j.max_helpers > 0)
      for (int i = 0; i < kJobSlots && slot < 0; i++) {
        Job* e = nullptr;
        if (jobs_[i].compare_exchange_strong(e, &j)) slot = i;
      }
    if (slot >= 0) {
      gen_.fetch_add(1);
      const int sleeping = sleepers_.load();
      if (sleeping > 0) {
        // wake what the job can use beyond the workers already spinning
        const int want = (int)std::min<size_t>(pieces - 1, (size_t)j.max_helpers) - spinning_.load();
        if (want > 0) {
          std::lock_guard<std::mutex> l(mu_);
          for (int k = 0; k < std::min(want, sleeping); k++) work_cv_.notify_one();
        }
      }
    }
    t_in_pool = true;
    work_on(&j);  // the caller's share (all of it when no slot was free)
    t_in_pool = false;
    if (slot < 0) return;
    jobs_[slot].store(nullptr);  // (no worker takes it from here on)
    // the pieces still running elsewhere (a spin of up to spin_us(), then
    // short sleeps: a long piece does not cost the caller a core), and the
    // workers that may still read j
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; j.finished.load(std::memory_order_acquire) != pieces; i++) {
      _mm_pause();
      if ((i & 63u) == 0 &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >= spin_us())
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    const int nw = nworkers_.load(std::memory_order_acquire);
    for (int w = 0; w < nw; w++)
      for (uint32_t i = 1; hazard_[w].load() == &j; i++) {
        _mm_pause();
        if ((i & 1023u) == 0) std::this_thread::yield();
      }
  }
  int threads() {
    start();
    return nworkers_.load();
  }
  // Testing: the most jobs that had pieces running at once since the last
  // call (counted from the first call on).
  int take_peak() {
    track_.store(true);
    return active_max_.exchange(0);
  }

 private:
  void work_on(Job* j) {
    for (;;) {
      const size_t k = j->next.fetch_add(1, std::memory_order_relaxed);
      if (k >= j->pieces) return;
      const bool track = track_.load(std::memory_order_relaxed);  // (tests only: shared counters)
      if (track && j->active.fetch_add(1) == 0) {
        const int r = running_.fetch_add(1) + 1;
        int m = active_max_.load();
        while (r > m && !active_max_.compare_exchange_weak(m, r)) {
        }
      }
      (*j->fn)(k);
      if (track && j->active.fetch_sub(1) == 1) running_.fetch_sub(1);
      j->finished.fetch_add(1, std::memory_order_release);
    }
  }
  // q (held by hazard slot w) has pieces left and room for one more helper:
  // join it.
  static bool join(Job* q) {
    if (q->next.load(std::memory_order_relaxed) >= q->pieces) return false;
    if (q->helpers.load(std::memory_order_relaxed) >= q->max_helpers) return false;
    if (q->helpers.fetch_add(1) < q->max_helpers) return true;
    q->helpers.fetch_sub(1);
    return false;
  }
  // A published job this worker may join, preferring this node's: held by
  // hazard slot w on return (nullptr: none).
  Job* take(int w, int node) {
    Job* any = nullptr;
    int any_i = -1;
    for (int i = 0; i < kJobSlots; i++) {
      Job* q = jobs_[i].load(std::memory_order_acquire);
      if (!q) continue;
      hazard_[w].store(q);
      if (jobs_[i].load() != q || q->next.load(std::memory_order_relaxed) >= q->pieces ||
          q->helpers.load(std::memory_order_relaxed) >= q->max_helpers) {
        hazard_[w].store(nullptr);
        continue;
      }
      const bool mine = q->node == node;  // (read while the hazard holds q)
      if (mine && join(q)) return q;      // (held)
      hazard_[w].store(nullptr);
      if (!any && !mine) {
        any = q;
        any_i = i;
      }
    }
    if (any) {  // another node's job: take it again under the hazard
      hazard_[w].store(any);
      if (jobs_[any_i].load() == any && join(any)) return any;
      hazard_[w].store(nullptr);
    }
    return nullptr;
  }
  void start() {
    if (started_.load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> l(mu_);
    if (started_.load(std::memory_order_relaxed)) return;
    const std::vector<NodeCpus> nodes = process_nodes();
    const int total = std::min(kMaxWorkers, std::max(1, usable_cores() - 1));  // (the caller is the last core)
    size_t cpus = 0;
    for (const NodeCpus& n : nodes) cpus += n.cpus.size();
    const bool bind = nodes.size() > 1;
    int given = 0;
    for (size_t i = 0; i < nodes.size(); i++) {
      // workers in proportion to the node's CPUs (at least one per node)
      const int left = total - given;
      int k = i + 1 == nodes.size()
                  ? left
                  : std::max(1, (int)((double)total * nodes[i].cpus.size() / std::max<size_t>(1, cpus) + 0.5));
      k = std::max(0, std::min(k, left));
      for (int t = 0; t < k; t++) {
        const int node = nodes[i].node, w = given + t;
        std::thread th([this, node, bind, w] { worker(w, node, bind); });
        th.detach();  // for the life of the process
      }
      given += k;
    }
    nworkers_.store(given, std::memory_order_release);
    started_.store(true, std::memory_order_release);
  }
  // How long a worker that found nothing spins for the next publication
  // before it sleeps (LSBM_POOL_SPIN_US, default 20): a staged table's four
  // chunk copies come back to back, and a worker still spinning joins the
  // next one at once; every microsecond of it is host CPU the database's own
  // threads do not get.
  static double spin_us() {
    static const double us = [] {
      const char* v = getenv("LSBM_POOL_SPIN_US");
      return v ? std::max(0.0, atof(v)) : 20.0;
    }();
    return us;
  }
  void worker(int w, int node, bool bind) {
    t_in_pool = true;
    NumaBind nb(bind ? node : -1, true, false);  // (kept bound for the thread's life)
    for (;;) {
      const uint64_t g = gen_.load();  // (before the look: a later publication changes it)
      Job* j = take(w, node);
      if (j) {
        work_on(j);
        hazard_[w].store(nullptr);  // (j may be gone after this)
        continue;
      }
      idle(g);
    }
  }
  // Until a publication after generation g: a bounded spin, then sleep.
  void idle(uint64_t g) {
    spinning_.fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    bool moved = false;
    for (uint32_t i = 1; !(moved = gen_.load(std::memory_order_acquire) != g); i++) {
      _mm_pause();
      if ((i & 63u) == 0 &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >= spin_us())
        break;
    }
    spinning_.fetch_sub(1);
    if (moved) return;
    std::unique_lock<std::mutex> l(mu_);
    sleepers_.fetch_add(1);
    work_cv_.wait(l, [&] { return gen_.load() != g; });
    sleepers_.fetch_sub(1);
  }
  std::mutex mu_;  // start() and sleeping only
  std::condition_variable work_cv_;
  std::atomic<Job*> jobs_[kJobSlots] = {};
  std::atomic<Job*> hazard_[kMaxWorkers] = {};
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> sleepers_{0}, spinning_{0}, nworkers_{0};
  std::atomic<bool> started_{false};
  std::atomic<int> running_{0}, active_max_{0};
  std::atomic<bool> track_{false};
};

WorkPool* pool() {
  static WorkPool* p = new WorkPool;  // never destroyed: its threads outlive static teardown
  return p;
}

constexpr int kMaxDevices = 64;

// Sessions of each device: leased one per caller, created on demand up to
// max_sessions(), kept for reuse (their pinned staging stays allocated).
struct DeviceSessions {
  std::vector<HostSession*> all, idle;
  std::condition_variable cv;
};
std::mutex g_reg;
DeviceSessions g_sessions[kMaxDevices];

int max_sessions() {
  static const int n = [] {
    const char* v = getenv("LSBM_HOST_SESSIONS");
    const int k = v ? atoi(v) : 0;
    return k > 0 ? std::min(k, 64) : 8;
  }();
  return n;
}

}  // namespace

void parallel_for(size_t pieces, const std::function<void(size_t)>& fn, int max_helpers) {
  if (pieces == 1 || (pieces > 1 && (t_in_pool || max_helpers == 0))) {  // (nested: inline on this worker)
    for (size_t k = 0; k < pieces; k++) fn(k);
    return;
  }
  if (pieces > 1) pool()->run(pieces, fn, t_job_node, max_helpers);
}

// One thread copies ~50 GB/s into pinned staging with non-temporal stores
// (profiles/r04/check18/one_auto_p1.log:3) and PCIe takes ~56 GB/s: the caller
// and 3 workers keep the copy well ahead of the DMA (LSBM_COPY_THREADS, the
// threads in all, caller included).  Round 4 used every pool thread (a 170
// GB/s burst for the first 4 MiB share, and every core of the quota busy).
int copy_helpers() {
  static const int n = [] {
    const char* v = getenv("LSBM_COPY_THREADS");
    const int t = v ? atoi(v) : 4;
    return std::max(0, std::min(t > 0 ? t : 4, pool()->threads() + 1) - 1);
  }();
  return n;
}

int pool_threads() { return pool()->threads(); }
int pool_take_peak_jobs() { return pool()->take_peak(); }

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

// Pieces of about n / (2 (helpers + 1)), at least 128 KiB, 4 KiB multiples,
// over the caller and copy_helpers() workers.
void parallel_copy(void* dst, const void* src, size_t n) {
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  constexpr size_t kMinPiece = 128u << 10;
  if (n < 2 * kMinPiece || t_in_pool) {
    stream_copy(d, s, n);
    return;
  }
  const int helpers = copy_helpers();
  const size_t ways = 2 * ((size_t)helpers + 1);
  const size_t piece = std::max(kMinPiece, ((n + ways - 1) / ways + 4095) / 4096 * 4096);
  parallel_for(
      (n + piece - 1) / piece,
      [&](size_t k) {
        const size_t off = k * piece;
        stream_copy(d + off, s + off, std::min(piece, n - off));
      },
      helpers);
}

// ---- per-call page locks ----
bool CallLocks::enabled() {
  static const bool on = [] {
    const char* e = getenv("LSBM_AUTO_LOCK");
    return !e || atoi(e) != 0;
  }();
  return on;
}

bool CallLocks::add(int device, const void* p, size_t n, bool writable) {
  static int read_only[kMaxDevices];  // 0 unknown, 1 supported, 2 not
  if (!p || n == 0 || device < 0 || device >= kMaxDevices) return false;
  if (__atomic_load_n(&read_only[device], __ATOMIC_RELAXED) == 0) {
    hipDeviceProp_t prop;
    const int v = hipGetDeviceProperties(&prop, device) == hipSuccess && prop.hostRegisterReadOnlySupported ? 1 : 2;
    __atomic_store_n(&read_only[device], v, __ATOMIC_RELAXED);
  }
  const bool ro = __atomic_load_n(&read_only[device], __ATOMIC_RELAXED) == 1;
  if (!ro && !writable) return false;
  const uintptr_t lo = page_lo(p), hi = page_hi(p, n);
  // The check and a reservation of the range's pages are one step against
  // every other call's locks (under g_lock_mu); the registration itself, which
  // pins the pages (~1-2 ms for 16 MiB of fresh pageable memory), runs outside
  // the mutex, so that callers on disjoint images lock them in parallel, while
  // a reserved range keeps every other call from registering or counting as
  // page-locked any page it touches until this call has unlocked it.
  // (Registration under the mutex serialised 4 concurrent 16 MiB callers to
  // 0.8x of running them one after another.)
  {
    std::lock_guard<std::mutex> l(g_lock_mu);
    if (touches_locked(lo, hi)) return false;  // (another live call's pages: staged)
    // Never over a registration the caller made: HIP accepts a range whose
    // first page is registered already, and unregistering such a range can
    // break the older one (a crash in a later call, found by table_gpu_test).
    // Both ends must be unregistered memory; a registration strictly inside
    // the range makes hipHostRegister fail.
    auto registered = [](const void* x) {
      hipPointerAttribute_t a;
      const hipError_t e = hipPointerGetAttributes(&a, x);
      (void)hipGetLastError();
      return e == hipSuccess && a.type != hipMemoryTypeUnregistered;
    };
    if (registered(p) || registered(static_cast<const char*>(p) + n - 1)) return false;
    g_locked.emplace(lo, hi);  // reserved
  }
  auto unreserve = [&] {
    std::lock_guard<std::mutex> l(g_lock_mu);
    g_locked.erase(lo);
  };
  void* q = const_cast<void*>(p);
  if (hipHostRegister(q, n, ro ? hipHostRegisterReadOnly : hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();  // (e.g. a registration inside the range)
    unreserve();
    return false;
  }
  // A range that shares its first page with an older registration registers,
  // but HIP then resolves its first byte to the older one, and an async DMA of
  // the whole range fails: only a range that now resolves as one buffer from
  // end to end counts (the staging copy takes the rest).
  if (!pinned_range(p, n)) {
    (void)hipHostUnregister(q);
    (void)hipGetLastError();
    unreserve();
    return false;
  }
  regs_.push_back(Reg{q, lo});
  g_locks_taken.fetch_add(1);
  return true;
}

CallLocks::~CallLocks() {
  if (regs_.empty()) return;
  // unlock first, then release the reservations: no other call touches the
  // pages until they are unregistered
  for (const Reg& r : regs_) (void)hipHostUnregister(r.p);
  (void)hipGetLastError();
  std::lock_guard<std::mutex> l(g_lock_mu);
  for (const Reg& r : regs_) g_locked.erase(r.lo);
}

// ---- buffers ----
// Page-locked host memory on `node` (the device's NUMA node): the pages are
// placed by the allocating thread's policy (hipHostMallocNumaUser) set to
// "prefer node" for the call; without NUMA information, HIP's default.
static hipError_t host_alloc(void** p, size_t bytes, unsigned flags, int node) {
  NumaBind nb(node, false, true);
  return hipHostMalloc(p, bytes, flags | (nb.memory_bound() ? hipHostMallocNumaUser : 0));
}

// A buffer grows to the size asked for plus a quarter (1 MiB granules), so
// that a session sized by one table's 4 MiB chunks pins ~5 MiB per stage, not
// a compaction's 80 MiB (a new session pinned 4 x 80 MiB: ~0.3 s), and grows
// once when larger jobs come.
static size_t with_headroom(size_t bytes) {
  bytes = std::max<size_t>(bytes, 1u << 16);
  if (bytes < (1u << 20)) return bytes;
  return (bytes + bytes / 4 + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
}

// Page-locked bytes held by each device's sessions, and the budget above which
// a released lease trims the idle sessions' staging (LSBM_PINNED_MB per
// device, default 1024): up to 8 sessions x 4 stages of compaction-sized
// buffers (~80 MiB each) would otherwise pin ~2.5 GiB per device until
// shutdown.  A failed allocation trims every idle session of the
// device and tries once more before the call fails.
namespace {
std::atomic<size_t> g_pinned[kMaxDevices];

size_t pinned_budget() {
  static const size_t b = [] {
    const char* v = getenv("LSBM_PINNED_MB");
    const long mb = v ? atol(v) : 1024;
    return (size_t)std::max(0L, mb) << 20;
  }();
  return b;
}

void count_pinned(int device, long long delta) {
  if (device >= 0 && device < kMaxDevices) g_pinned[device].fetch_add((size_t)delta);
}

// Frees the staging of the device's idle sessions but the `keep` most
// recently released (under g_reg; an idle session has no work in flight:
// its lease drained every stage).
void trim_idle_locked(int device, size_t keep) {
  DeviceSessions& ds = g_sessions[device];
  for (size_t i = 0; i + keep < ds.idle.size(); i++) ds.idle[i]->release_staging();
}
}  // namespace

// Registrations through lsbm_host_register: within the same LSBM_PINNED_MB
// (all of them together, whichever device DMAs from them).
size_t host_register_budget() { return pinned_budget(); }

size_t pinned_bytes(int device) {
  return device >= 0 && device < kMaxDevices ? g_pinned[device].load() : 0;
}

hipError_t StagePair::alloc(size_t bytes, bool map) {
  bytes = with_headroom(bytes);
  hipError_t e = hipSuccess;
  for (int attempt = 0; attempt < 2; attempt++) {
    if (attempt) {  // (pinned or device memory ran out: give back the idle sessions' staging)
      if (device < 0 || device >= kMaxDevices) break;
      std::lock_guard<std::mutex> l(g_reg);
      trim_idle_locked(device, 0);
    }
    e = host_alloc(reinterpret_cast<void**>(&h), bytes,
                   map ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault, node);
    if (e == hipSuccess) {
      count_pinned(device, (long long)bytes);
      cap = bytes;  // (release() uncounts it from here on)
      mapped = map;
      e = map ? hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0)
              : hipMalloc(reinterpret_cast<void**>(&d), bytes);
    }
    if (e == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    release();
  }
  return e;
}

hipError_t StagePair::reserve(size_t bytes) {
  if (bytes <= cap && !mapped) return hipSuccess;
  release();
  return alloc(bytes, false);
}

hipError_t StagePair::reserve_mapped(size_t bytes) {
  if (bytes <= cap && mapped) return hipSuccess;
  release();
  return alloc(bytes, true);
}

void StagePair::release() {
  if (h) {
    (void)hipHostFree(h);
    count_pinned(device, -(long long)cap);
  }
  if (d && !mapped) (void)hipFree(d);
  h = d = nullptr;
  cap = 0;
  mapped = false;
}

void HostSession::release_staging() {
  DeviceGuard g(device_);
  for (Stage& s : stage_) {
    s.bulk.release();
    s.meta.release();
    s.res.release();
    s.zmeta.release();
  }
}

// ---- session ----
// How a caller waits for its stage (HostSession::wait): spinning in
// hipEventSynchronize (the default: the lowest latency, a core busy for the
// call), or, LSBM_BLOCKING_WAIT=1, sleeping on a blocking-sync event.
bool blocking_wait() {
  static const bool b = [] {
    const char* v = getenv("LSBM_BLOCKING_WAIT");
    return v && atoi(v) != 0;
  }();
  return b;
}

hipError_t HostSession::init() {
  node_ = device_numa_node(device_);
  for (Stage& s : stage_) {
    s.bulk.node = s.meta.node = s.res.node = s.zmeta.node = node_;
    s.bulk.device = s.meta.device = s.res.device = s.zmeta.device = device_;
    hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess)
      e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming | (blocking_wait() ? hipEventBlockingSync : 0u));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.copied, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

HostSession::~HostSession() {
  DeviceGuard g(device_);
  if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
  for (Stage& s : stage_) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.bulk.release();
    s.meta.release();
    s.res.release();
    s.zmeta.release();
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
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

hipError_t HostSession::copy_stream(hipStream_t* out) {
  if (!copy_stream_) {
    const hipError_t e = hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking);
    if (e != hipSuccess) {
      copy_stream_ = nullptr;
      return e;
    }
  }
  copy_pending_ = true;
  *out = copy_stream_;
  return hipSuccess;
}

// A stage's wait.  hipEventSynchronize spins for the whole wait on this
// runtime, with or without hipEventBlockingSync (tools/probe_wait.cc,
// profiles/r05/host_cpu/probe_wait.log: 0.30 ms of the caller's CPU per 0.31 ms
// wait either way), so a one-table call cost a core for its whole 0.35 ms.
// By default the caller now sleeps in short naps, polling the event, until
// the stage's expected wait (a moving average of its previous ones) is within
// kSpinMarginUs, and only then spins: the call's CPU drops to the margin plus
// the polls while its latency stays that of the spin.  LSBM_WAIT=spin keeps
// the plain spin.
namespace {
constexpr double kSpinMarginUs = 60.0;
bool hybrid_wait() {
  static const bool h = [] {
    const char* v = getenv("LSBM_WAIT");
    return !(v && strcmp(v, "spin") == 0) && !blocking_wait();
  }();
  return h;
}
double us_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

hipError_t HostSession::wait(Stage& s) {
  if (!s.busy) return hipSuccess;
  s.busy = false;
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipSuccess;
  bool done = false;
  if (hybrid_wait() && s.wait_ewma_us > kSpinMarginUs) {
    const double sleep_until = s.wait_ewma_us - kSpinMarginUs;
    for (double el = 0; el < sleep_until; el = us_since(t0)) {
      const hipError_t q = hipEventQuery(s.done);
      if (q == hipSuccess) {
        done = true;
        break;
      }
      if (q != hipErrorNotReady) {
        e = q;
        break;
      }
      const double nap = std::min(20.0, sleep_until - el);
      std::this_thread::sleep_for(std::chrono::microseconds((long)nap + 1));
    }
    (void)hipGetLastError();  // (the polls' "not ready")
  }
  if (!done && e == hipSuccess) e = hipEventSynchronize(s.done);
  const double took = us_since(t0);
  s.wait_ewma_us = s.wait_ewma_us == 0 ? took : 0.75 * s.wait_ewma_us + 0.25 * took;
  s.settled = e == hipSuccess;
  return e;
}

hipError_t HostSession::upload(void* d, const void* h, size_t n) {
  if (n == 0) return hipSuccess;
  if (host_pinned(h, n)) {
    Stage& s0 = stage_[0];
    for (Stage& s : stage_) s.settled = false;
    hipError_t e = hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s0.stream);
    return e == hipSuccess ? hipStreamSynchronize(s0.stream) : e;
  }
  const Piece one = {h, n};
  return upload_pieces(d, &one, 1);
}

hipError_t HostSession::upload_pieces(void* d, const Piece* pieces, size_t count) {
  size_t n = 0;
  for (size_t p = 0; p < count; p++) n += pieces[p].n;
  if (n == 0) return hipSuccess;
  Stage& s0 = stage_[0];
  for (Stage& s : stage_) s.settled = false;
  // through the stages' pinned buffers: stage i's copy overlaps stage i-1's
  // DMA (on the other stages' streams, so stage 0's queue is drained first)
  hipError_t e0 = hipStreamSynchronize(s0.stream);
  if (e0 != hipSuccess) return e0;
  int i = 0;
  size_t p = 0, in_p = 0;  // the next byte to stage: piece p, offset in_p
  for (size_t off = 0; off < n; off += kChunkBytes, i = (i + 1) % kStages) {
    const size_t k = std::min(kChunkBytes, n - off);
    Stage& s = stage_[i];
    hipError_t e = wait(s);
    if (e == hipSuccess) e = s.bulk.reserve(kChunkBytes);
    if (e != hipSuccess) return e;
    for (size_t filled = 0; filled < k;) {  // the chunk from the pieces it spans
      while (in_p == pieces[p].n) p++, in_p = 0;
      const size_t take = std::min(k - filled, pieces[p].n - in_p);
      parallel_copy(s.bulk.h + filled, static_cast<const char*>(pieces[p].h) + in_p, take);
      filled += take;
      in_p += take;
    }
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
  for (Stage& s : stage_) s.settled = false;
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
  std::unique_lock<std::mutex> l(g_reg);
  for (int dev = 0; dev < kMaxDevices; dev++) {
    DeviceSessions& ds = g_sessions[dev];
    ds.cv.wait(l, [&] { return ds.idle.size() == ds.all.size(); });  // no lease may be open
    for (HostSession* s : ds.all) delete s;
    ds.all.clear();
    ds.idle.clear();
  }
}

// ---- lease ----
// Every exit path of a layer (an error between enqueueing a chunk and
// collecting it included) ends here: the stages' work is waited for and their
// results dropped, so that no later call collects a stale chunk (its tag would
// index that call's plan) and no DMA from the caller's memory is still in
// flight when the layer returns.
SessionLease::~SessionLease() {
  if (s_) {
    bool all_settled = true;
    for (int i = 0; i < HostSession::kStages; i++) {
      Stage& sg = s_->stage(i);
      all_settled = all_settled && sg.settled && !sg.busy;
      if (sg.stream && !(sg.settled && !sg.busy)) (void)hipStreamSynchronize(sg.stream);
      sg.busy = false;
      sg.settled = false;
    }
    // The copy stream's DMAs all precede a stage's kernel (stream-wait on the
    // stage's `copied` event), so settled stages mean finished copies; on an
    // error path one may still be reading the caller's memory.
    if (s_->copy_stream_ && s_->copy_pending_ && !all_settled) (void)hipStreamSynchronize(s_->copy_stream_);
    s_->copy_pending_ = false;
    std::lock_guard<std::mutex> l(g_reg);
    DeviceSessions& ds = g_sessions[s_->device()];
    ds.idle.push_back(s_);
    if (pinned_bytes(s_->device()) > pinned_budget()) trim_idle_locked(s_->device(), 1);
    ds.cv.notify_all();
  }
  if (node_set_) t_job_node = prev_node_;  // (only what Open set: an outer lease's node stays)
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

// A session of `device` for this caller: an idle one, else a new one while
// the device has fewer than max_sessions(), else the next one released.
// Concurrent callers on one device (the reference's writer, compaction and
// reader threads) each get their own stages and streams and run at once.
Status SessionLease::Open(int device) {
  if (device < 0 || device >= kMaxDevices) return Status::InvalidArgument("bad device ordinal");
  if (lsbm_crc32c_init(device) != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
  guard_ = new DeviceGuard(device);
  if (guard_->status() != hipSuccess) return hip_status(guard_->status(), "hipSetDevice");
  HostSession* s = nullptr;
  bool fresh = false;
  {
    std::unique_lock<std::mutex> l(g_reg);
    DeviceSessions& ds = g_sessions[device];
    ds.cv.wait(l, [&] { return !ds.idle.empty() || (int)ds.all.size() < max_sessions(); });
    if (!ds.idle.empty()) {
      s = ds.idle.back();
      ds.idle.pop_back();
    } else {
      s = new HostSession(device);
      ds.all.push_back(s);  // (counted now, so that concurrent opens respect the cap)
      fresh = true;
    }
  }
  if (fresh) {
    const hipError_t e = s->init();  // streams on `device` (current)
    if (e != hipSuccess) {
      std::lock_guard<std::mutex> l(g_reg);
      DeviceSessions& ds = g_sessions[device];
      ds.all.erase(std::find(ds.all.begin(), ds.all.end(), s));
      delete s;
      ds.cv.notify_all();
      return hip_status(e, "session streams");
    }
  }
  s_ = s;
  prev_node_ = t_job_node;
  node_set_ = true;
  t_job_node = s->node();
  return Status::OK();
}

int session_count(int device) {
  if (device < 0 || device >= kMaxDevices) return 0;
  std::lock_guard<std::mutex> l(g_reg);
  return (int)g_sessions[device].all.size();
}

}  // namespace lsbm

// Testing only (include/lsbm_crc32c.h): the next host-layer pipeline fails
// once it has enqueued `chunks` chunks (-1: off).
extern "C" __attribute__((visibility("default"))) int lsbm_test_fail_host_pipeline(int chunks) {
  lsbm::g_fault_after.store(chunks < 0 ? -1 : chunks);
  return 0;
}

extern "C" __attribute__((visibility("default"))) int lsbm_host_threads(void) {
  return lsbm::pool_threads();
}

extern "C" __attribute__((visibility("default"))) int lsbm_test_pool_overlap(int callers, int jobs, int pieces,
                                                                         int piece_us, double* seconds) {
  if (callers <= 0 || jobs <= 0 || pieces <= 0 || piece_us < 0) return -1;
  (void)lsbm::pool_take_peak_jobs();
  const double t0 = lsbm::HostTiming::now();
  std::vector<std::thread> th;
  for (int c = 0; c < callers; c++)
    th.emplace_back([=] {
      for (int j = 0; j < jobs; j++)
        lsbm::parallel_for((size_t)pieces,
                           [=](size_t) { std::this_thread::sleep_for(std::chrono::microseconds(piece_us)); });
    });
  for (auto& t : th) t.join();
  if (seconds) *seconds = lsbm::HostTiming::now() - t0;
  return lsbm::pool_take_peak_jobs();
}

// Testing: `callers` threads each run `jobs` parallel_for jobs of 1..max_pieces
// pieces (helper caps from none to 3 or any; some nested: a piece that runs
// its own parallel_for, inline), each
// piece adding 1 to its own counter; returns the number of counters that
// are not exactly 1 afterwards (0: every piece of every job ran once).
extern "C" __attribute__((visibility("default"))) int lsbm_test_pool_stress(int callers, int jobs, int max_pieces) {
  if (callers <= 0 || jobs <= 0 || max_pieces <= 0) return -1;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int c = 0; c < callers; c++)
    th.emplace_back([=, &bad] {
      uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1);
      for (int j = 0; j < jobs; j++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        const size_t n = 1 + (size_t)(x % (uint64_t)max_pieces);
        std::vector<std::atomic<int>> hit(n);
        for (auto& h : hit) h.store(0);
        const bool nested = (x >> 40) % 5 == 0;
        const int cap = (int)((x >> 20) % 5) - 1;  // helper caps -1 (any) .. 3
        lsbm::parallel_for(
            n,
            [&](size_t k) {
              if (nested) {
                std::atomic<int> inner{0};
                lsbm::parallel_for(3, [&](size_t) { inner.fetch_add(1); });
                if (inner.load() != 3) hit[k].fetch_add(100);
              }
              hit[k].fetch_add(1);
            },
            cap);
        for (auto& h : hit) bad += h.load() != 1;
      }
    });
  for (auto& t : th) t.join();
  return bad.load();
}

// Testing: host_pinned() itself (which ranges the layers DMA in place).
extern "C" __attribute__((visibility("default"))) int lsbm_test_host_copy(void* dst, const void* src, size_t n,
                                                                      int parallel) {
  if (parallel)
    lsbm::parallel_copy(dst, src, n);
  else
    lsbm::stream_copy(static_cast<char*>(dst), static_cast<const char*>(src), n);
  return 0;
}

extern "C" __attribute__((visibility("default"))) int lsbm_test_host_pinned(const void* p, size_t n) {
  return lsbm::host_pinned(p, n) ? 1 : 0;
}

// Testing: how many distinct threads ran the pieces of one capped job.
extern "C" __attribute__((visibility("default"))) int lsbm_test_pool_helpers(int pieces, int piece_us,
                                                                         int max_helpers) {
  if (pieces <= 0 || piece_us < 0) return -1;
  std::mutex mu;
  std::vector<std::thread::id> ids;
  lsbm::parallel_for(
      (size_t)pieces,
      [&](size_t) {
        {
          std::lock_guard<std::mutex> l(mu);
          if (std::find(ids.begin(), ids.end(), std::this_thread::get_id()) == ids.end())
            ids.push_back(std::this_thread::get_id());
        }
        std::this_thread::sleep_for(std::chrono::microseconds(piece_us));
      },
      max_helpers);
  return (int)ids.size();
}

extern "C" __attribute__((visibility("default"))) int lsbm_host_register(const void* p, uint64_t n) {
  return lsbm::host_register(p, (size_t)n);
}

extern "C" __attribute__((visibility("default"))) int lsbm_host_unregister(const void* p) {
  return lsbm::host_unregister(p);
}

extern "C" __attribute__((visibility("default"))) unsigned long long lsbm_host_registered_bytes(void) {
  return (unsigned long long)lsbm::host_registered_bytes();
}

extern "C" __attribute__((visibility("default"))) int lsbm_test_locked_ranges(void) {
  return lsbm::locked_ranges();
}

extern "C" __attribute__((visibility("default"))) long lsbm_test_locks_taken(void) {
  return lsbm::locks_taken();
}

// Testing: the C++ layers' sessions of `device` and the page-locked staging
// bytes they hold (the pinned budget, LSBM_PINNED_MB).
extern "C" __attribute__((visibility("default"))) int lsbm_test_session_count(int device) {
  return lsbm::session_count(device);
}

extern "C" __attribute__((visibility("default"))) unsigned long long lsbm_test_pinned_bytes(int device) {
  return (unsigned long long)lsbm::pinned_bytes(device);
}
