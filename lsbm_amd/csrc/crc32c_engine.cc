// crc32c_engine.cc -- the C ABI of include/lsbm_crc32c.h (host side).
//
// Owns the per-device tables (built once with std::call_once, then read-only),
// validates arguments, picks the kernel, and runs the host-staged pipeline.
// Never throws, never aborts, never computes a batch on the CPU: without a
// usable HIP device every batch entry point returns LSBM_ERR_NO_DEVICE.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsbm_crc32c.h"
#include "crc32c_types.h"
#include "engine_internal.h"
#include "gf2.h"
#include "host_numa.h"
#include "host_session.h"

namespace lsbm {

// launchers (crc32c_kernels.hip)
hipError_t launch_fixed(const uint8_t* base, uint64_t stride, uint32_t rows, uint64_t n_blocks,
                        const uint32_t* init, uint32_t* out, uint32_t flags, uint32_t k_value,
                        const DevConsts* dc, int grid, hipStream_t stream,
                        uint32_t* heads);
hipError_t launch_ragged(const RaggedArgs& a, int grid, hipStream_t stream);
bool ragged_uses_stream(const RaggedArgs& a);
int set_ragged_policy(int p);
hipError_t launch_range_bounds(const RaggedArgs& a, uint64_t P, uint32_t* bounds, int grid,
                               hipStream_t stream);
hipError_t launch_trailer_scatter(uint8_t* file, uint64_t limit, const uint64_t* handles, const uint8_t* types,
                                  const uint32_t* crcs, uint64_t n, int grid, hipStream_t stream);
hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, int grid, hipStream_t stream);
hipError_t launch_gather(const uint8_t* src, const uint64_t* src_off, const uint64_t* len, uint64_t n,
                         uint8_t* dst, const uint64_t* dst_off, int grid, hipStream_t stream);
hipError_t launch_stream_read(const void* buf, uint64_t nbytes, uint32_t* sink, int grid,
                              hipStream_t stream);

namespace {

thread_local char t_last_error[256] = "";

int fail_hip(hipError_t e, const char* what) {
  snprintf(t_last_error, sizeof(t_last_error), "%s: %s", what, hipGetErrorString(e));
  return LSBM_ERR_HIP;
}
int fail(int code, const char* what) {
  snprintf(t_last_error, sizeof(t_last_error), "%s", what);
  return code;
}

constexpr int kMaxDevices = 64;

// Per-device tables: built on first use, read-only until lsbm_crc32c_shutdown.
// `ready` is the lock-free fast path of every call; `mu` serialises the
// first initialisation (and shutdown) of a device.
struct DeviceState {
  std::mutex mu;
  std::atomic<bool> ready{false};
  int status = LSBM_ERR_NO_DEVICE;
  DevConsts* d_consts = nullptr;
  int num_cus = 0;
};
DeviceState g_dev[kMaxDevices];

void build_consts(DevConsts* c) {
  gf2::byte_tables(gf2::byte_pow(kRowBytes), c->row_byte);
  {
    uint32_t tmp[1024];
    gf2::byte_tables(gf2::byte_pow(1), tmp);
    memcpy(c->t0, tmp, sizeof(c->t0));  // M(b << 0) = A(b) = table0_[b]
  }
  gf2::Mat p = gf2::byte_pow(1);
  for (int k = 0; k < 64; k++) {
    gf2::nibble_tables(p, c->pow_nib[k]);
    p = gf2::mul(p, p);
  }
  // (powers built one step from the last, not each by squaring: the device's
  // set-up is then ~1 ms of host work instead of ~15)
  const gf2::Mat inv1 = gf2::byte_pow(-1), fwd1 = gf2::byte_pow(1);
  {
    gf2::Mat m = gf2::identity();
    for (int z = 0; z < 128; z++, m = gf2::mul(inv1, m)) gf2::nibble_tables(m, c->neg_nib[z]);
  }
  gf2::nibble_tables(gf2::byte_pow(-4), c->neg4_nib);
  for (int li = 0; li < 8; li++) gf2::nibble_tables(gf2::byte_pow(116 - 16 * li), c->fin_nib[li]);
  // LDS image (layout: crc32c_device.h header comment)
  memset(c->lds_image, 0, sizeof(c->lds_image));
#ifdef LSBM_LDS16
  {
    uint32_t a4[1024];
    gf2::byte_tables(gf2::byte_pow(4), a4);
    for (uint32_t w = 0; w < 0x10000 / 4; w++) {
      const uint32_t a = w << 2, t = (a >> 6) & 3u, b = (a >> 8) & 255u;
      c->lds_image[w] = c->row_byte[t * 256 + b];
      c->lds_image[kByteA4 / 4 + w] = a4[t * 256 + b];
    }
  }
#else
  for (uint32_t w = 0; w < kLdsByteTabBytes / 4; w++) {
    const uint32_t a = w << 2;
    const uint32_t t = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t b = (a >> 8) & 255u;
    c->lds_image[w] = c->row_byte[t * 256 + b];
  }
#endif
  for (uint32_t w = 0; w < 128; w++) c->lds_image[kNibA4 / 4 + w] = c->pow_nib[2][w];
  for (uint32_t w = 0; w < 128; w++) c->lds_image[kNibA8 / 4 + w] = c->pow_nib[3][w];
  gf2::nibble_tables(gf2::byte_pow(12), &c->lds_image[kNibA12 / 4]);
  for (uint32_t w = 0; w < 8 * 16 * 32; w++) {
    const uint32_t q = w >> 9, nib = (w >> 5) & 15u, slot = w & 31u;
    c->lds_image[kNibFin / 4 + w] = c->fin_nib[slot & 7u][q * 16 + nib];
  }
  for (uint32_t i = kRowPowLo; i < kRowPowTables; i++)  // A^(128 * 2^i) = A^(2^(7+i))
    memcpy(&c->lds_image[kNibRowPow / 4 + i * 128], c->pow_nib[7 + i], 512);
  for (uint32_t i = 0; i < 8; i++)  // A^(2^i) (stream kernel finish)
    memcpy(&c->lds_image[kNibPow2 / 4 + i * 128], c->pow_nib[i], 512);
  gf2::nibble_tables(gf2::byte_pow(-128), &c->lds_image[kNibNeg128 / 4]);
  memcpy(&c->lds_image[kNibNeg4 / 4], c->neg4_nib, 512);
  for (uint32_t lo = 0; lo <= 16; lo++)  // stream kernel: bytes [lo, hi) of a 16-B chunk
    for (uint32_t hi = lo; hi <= 16; hi++) {
      const uint32_t t = km_entry(lo, hi);
      for (uint32_t b = 0; b < 16; b++)
        if (b >= lo && b < hi) c->lds_image[kStreamHM / 4 + t * 4 + b / 4] |= 0xffu << (8 * (b % 4));
    }
  {
    uint32_t v = 0xffffffffu;  // stream kernel: ~0 injected d bytes before the row start
    for (uint32_t d = 0; d < 128; d++, v = gf2::apply(inv1, v)) c->lds_image[kStreamR0 / 4 + d] = v;
  }
  memset(c->zero16, 0, sizeof(c->zero16));
  // column forms for the units kernel: A^(128 k) and A^e, e = -127 .. 1
  {
    const gf2::Mat row = gf2::byte_pow(kRowBytes);
    gf2::Mat m = gf2::identity();
    for (uint32_t k = 0; k < kShiftCols; k++) {
      memcpy(c->shift_cols[k], m.col, sizeof(m.col));
      m = gf2::mul(row, m);
    }
    gf2::Mat f = gf2::byte_pow(-127);
    for (uint32_t i = 0; i < kFinCols; i++, f = gf2::mul(fwd1, f)) memcpy(c->fin_cols[i], f.col, sizeof(f.col));
  }
}

void init_device(int dev, DeviceState* st) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || dev < 0 || dev >= count) {
    st->status = LSBM_ERR_NO_DEVICE;
    return;
  }
  int prev = 0;
  hipGetDevice(&prev);
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) {
    st->status = fail_hip(e, "hipSetDevice");
    return;
  }
  int cus = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess || cus <= 0) cus = 256;
  DevConsts* h = new (std::nothrow) DevConsts;
  if (!h) {
    st->status = fail(LSBM_ERR_NOMEM, "host alloc");
    hipSetDevice(prev);
    return;
  }
  build_consts(h);
  DevConsts* d = nullptr;
  e = hipMalloc(&d, sizeof(DevConsts));
  if (e == hipSuccess) e = hipMemcpy(d, h, sizeof(DevConsts), hipMemcpyHostToDevice);
  delete h;
  if (e != hipSuccess) {
    st->status = fail_hip(e, "device tables");
    if (d) hipFree(d);
    hipSetDevice(prev);
    return;
  }
  // Stream-ordered scratch (lsbm_sst_seal_dev) comes from the device's
  // default pool; keep freed blocks in the pool so that a steady stream of
  // calls reuses them instead of returning memory to the driver each time.
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess && pool) {
    uint64_t keep = ~0ull;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
  (void)hipGetLastError();
  st->d_consts = d;
  st->num_cus = cus;
  st->status = LSBM_OK;
  hipSetDevice(prev);
}

int ensure_device(int dev, DeviceState** out) {
  if (dev < 0 || dev >= kMaxDevices) return fail(LSBM_ERR_NO_DEVICE, "bad device ordinal");
  DeviceState* st = &g_dev[dev];
  if (!st->ready.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> l(st->mu);
    if (!st->ready.load(std::memory_order_relaxed)) {
      init_device(dev, st);
      if (st->status != LSBM_OK) return st->status;
      st->ready.store(true, std::memory_order_release);
    }
  }
  *out = st;
  return LSBM_OK;
}

int current_device(DeviceState** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail(LSBM_ERR_NO_DEVICE, "no current HIP device");
  return ensure_device(dev, out);
}

// Blocks per launch of the fixed kernel for big batches
// (LSBM_FIXED_SPLIT_BLOCKS; 0 = one launch whatever the size).
uint64_t fixed_split_blocks() {
  static const uint64_t b = [] {
    const char* v = getenv("LSBM_FIXED_SPLIT_BLOCKS");
    return v ? (uint64_t)strtoull(v, nullptr, 10) : (uint64_t)(1u << 20);
  }();
  return b;
}

// The fixed kernel's cross-XCC work queue (crc32c_units.h WgQueue), OFF by
// default (LSBM_FIXED_QUEUE=1 or lsbm_test_fixed_queue: on).  It does what it
// is for -- the eight XCDs' waves end within 5% of the launch instead of 14%
// but the chip's aggregate read rate does not move (config 2 84.8% either
// way, config 3 +0.7 points, a 10M-block shard -1 point; DESIGN.md section
// 4): a statically split batch's fast XCDs finish early and the slow ones
// then get their bandwidth.  Only for launches of at least 4 groups per wave,
// and never while the stream is being captured into a graph (the heads are
// per-call scratch).
std::atomic<int> g_fixed_queue{-1};  // -1: not read yet; 0 off, 1 on (lsbm_test_fixed_queue)
bool fixed_queue_on() {
  int q = g_fixed_queue.load(std::memory_order_relaxed);
  if (q < 0) {
    const char* v = getenv("LSBM_FIXED_QUEUE");
    q = (v && v[0] == '1') ? 1 : 0;
    int expect = -1;
    if (!g_fixed_queue.compare_exchange_strong(expect, q)) q = expect;
  }
  return q == 1;
}

// SSTable trailer batches as claimed equal-count pieces (LSBM_SST_PIECES=1,
// lsbm_test_sst_pieces: A/B runs) or one range per wave (the default: in one
// process over one image, pieces ran 0.1-0.35 points slower, round 6,
// profiles/r06/events_ab/sst_pieces_inproc.log).
std::atomic<int> g_sst_pieces{-1};  // -1: not read yet
bool sst_pieces_on() {
  int q = g_sst_pieces.load(std::memory_order_relaxed);
  if (q < 0) {
    const char* v = getenv("LSBM_SST_PIECES");
    q = (v && v[0] == '1') ? 1 : 0;
    int expect = -1;
    if (!g_sst_pieces.compare_exchange_strong(expect, q)) q = expect;
  }
  return q == 1;
}

int grid_for(const DeviceState* st, uint64_t n_blocks) {
  const uint64_t groups = (n_blocks + 7) / 8;
  const uint64_t wgs = (groups + kWavesPerWg - 1) / kWavesPerWg;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(wgs, (uint64_t)st->num_cus));
}

// A^-4(~0): the virtual init bytes of crc32c::Value (init 0), see crc32c_kernels.hip
uint32_t u_noinit() {
  static const uint32_t u = gf2::apply(gf2::byte_pow(-4), 0xffffffffu);
  return u;
}

// One launch, no host sync.  A general batch (Out / Verify over offsets or
// extents) of at least kMinChunks chunks of kChunkBlocks blocks per wave is
// swept chunk by chunk (crc32c_units_kernel): a first small launch finds every
// wave's byte-balanced range in every chunk, into (nchunks * nwaves + 1) * 4
// bytes of stream-ordered scratch from the device's default pool (which
// lsbm_crc32c_init sets to keep freed memory).  Without that scratch, and
// while the stream is being captured into a graph, the batch goes as one
// range per wave.
int run_ragged_one(RaggedArgs a, hipStream_t stream) {
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  if (a.n == 0) return LSBM_OK;
  a.dc = st->d_consts;
  a.u_noinit = u_noinit();
  a.bounds = nullptr;
  a.nchunks = 0;
  a.piece_q = a.piece_r = 0;
  const uint64_t nwaves =
      (uint64_t)st->num_cus * (ragged_uses_stream(a) ? kStreamWavesPerWg : kWavesPerWg);
  // (LSBM_SWEEP_CHUNK_BLOCKS: A/B runs only; 0 = no chunked sweep)
  static const uint64_t chunk_blocks = [] {
    const char* v = getenv("LSBM_SWEEP_CHUNK_BLOCKS");
    return v ? strtoull(v, nullptr, 10) : (uint64_t)kChunkBlocks;
  }();
  uint32_t* bounds = nullptr;
  if (chunk_blocks > 0 && (a.mode == kModeOut || a.mode == kModeVerify) &&
      (a.extents == kExtOffsets || a.extents == kExtHandles) &&
      a.n >= (uint64_t)kMinChunks * chunk_blocks * nwaves && a.n < 0xffffffffull) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const uint64_t nchunks = a.n / (chunk_blocks * nwaves);
    const uint64_t P = nchunks * nwaves;
    if (hipStreamIsCapturing(stream, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone &&
        hipMallocAsync(reinterpret_cast<void**>(&bounds), (P + 1) * sizeof(uint32_t), stream) ==
            hipSuccess) {
      const hipError_t e = launch_range_bounds(a, P, bounds, (int)st->num_cus * 8, stream);
      if (e != hipSuccess) {
        (void)hipFreeAsync(bounds, stream);
        return fail_hip(e, "range_bounds_kernel");
      }
      a.bounds = bounds;
      a.nchunks = nchunks;
    } else {
      (void)hipGetLastError();  // (no scratch: one range per wave)
      bounds = nullptr;
    }
  }
  // SSTable trailer batches (verify, dense trailer CRCs; not the fused seal,
  // whose trailer epilogue walks the wave's one range): equal-count pieces of
  // kSstPieceBlocks blocks, claimed by the workgroup's waves in turn
  // (crc32c_units.h next_piece), no bounds table.
  if (sst_pieces_on() && !bounds && a.extents == kExtHandles &&
      (a.mode == kModeSstVerify || (a.mode == kModeSstCrc && !a.file)) && a.n < 0xffffffffull) {
    const uint64_t per_wave = a.n / ((uint64_t)kSstPieceBlocks * nwaves);
    if (per_wave >= 2) {
      const uint64_t P = per_wave * nwaves;
      a.nchunks = per_wave;
      a.piece_q = (uint32_t)(a.n / P);
      a.piece_r = (uint32_t)(a.n % P);
    }
  }
  const hipError_t e = launch_ragged(a, (int)st->num_cus, stream);
  if (bounds) (void)hipFreeAsync(bounds, stream);
  return e == hipSuccess ? LSBM_OK : fail_hip(e, "crc32c_units_kernel");
}

// A big offsets batch (CRCs out) as back-to-back launches of
// LSBM_RAGGED_SPLIT_BLOCKS blocks (0, the default: one launch; A/B, DESIGN.md
// section 6 for the fixed-stride case).
int run_ragged(RaggedArgs a, hipStream_t stream) {
  static const uint64_t per = [] {
    const char* v = getenv("LSBM_RAGGED_SPLIT_BLOCKS");
    return v ? (uint64_t)strtoull(v, nullptr, 10) : (uint64_t)0;
  }();
  if (!(per && a.mode == kModeOut && a.extents == kExtOffsets && a.n >= 2 * per))
    return run_ragged_one(a, stream);
  for (uint64_t f = 0; f < a.n;) {
    const uint64_t m = a.n - f >= 2 * per ? per : a.n - f;
    RaggedArgs b = a;
    b.offsets = a.offsets + f;
    b.n = m;
    b.out = a.out + f;
    if (a.init) b.init = a.init + f;
    const int rc = run_ragged_one(b, stream);
    if (rc != LSBM_OK) return rc;
    f += m;
  }
  return LSBM_OK;
}

}  // namespace

// Testing (include/lsbm_crc32c.h): the fixed kernel's cross-XCC queue on (1)
// or off (0: the static interleave); -1 back to LSBM_FIXED_QUEUE's default.
extern "C" __attribute__((visibility("default"))) int lsbm_test_fixed_queue(int on) {
  if (on < -1 || on > 1) return -1;
  g_fixed_queue.store(on);
  return 0;
}

// Testing (include/lsbm_crc32c.h): SSTable trailer pieces on (1) or off (0);
// -1 back to LSBM_SST_PIECES's default.
extern "C" __attribute__((visibility("default"))) int lsbm_test_sst_pieces(int on) {
  if (on < -1 || on > 1) return -1;
  g_sst_pieces.store(on);
  return 0;
}

// engine_internal.h: shared with the bloom entry points (bloom_engine.cc)
int engine_fail(int code, const char* what) { return fail(code, what); }
int engine_fail_hip(hipError_t e, const char* what) { return fail_hip(e, what); }
int engine_current_cus(int* cus) {
  DeviceState* st = nullptr;
  const int rc = current_device(&st);
  if (rc == LSBM_OK) *cus = st->num_cus;
  return rc;
}

}  // namespace lsbm

using namespace lsbm;

extern "C" {

__attribute__((visibility("default"))) const char* lsbm_crc32c_version(void) {
  return "lsbm-crc32c-mi355x 0.1 (gfx950)";
}

__attribute__((visibility("default"))) const char* lsbm_crc32c_last_error(void) {
  return t_last_error;
}

__attribute__((visibility("default"))) int lsbm_crc32c_init(int device) {
  DeviceState* st = nullptr;
  return ensure_device(device, &st);
}

__attribute__((visibility("default"))) int lsbm_crc32c_shutdown(void) {
  // the sessions' staging first (it synchronises their streams), then the
  // per-device tables
  HostSession::ShutdownAll();
  int prev = 0;
  const bool have_prev = hipGetDevice(&prev) == hipSuccess;
  int rc = LSBM_OK;
  for (int dev = 0; dev < kMaxDevices; dev++) {
    DeviceState* st = &g_dev[dev];
    std::lock_guard<std::mutex> l(st->mu);
    if (!st->ready.load()) continue;
    if (hipSetDevice(dev) != hipSuccess) {
      rc = fail(LSBM_ERR_HIP, "hipSetDevice");
      continue;
    }
    (void)hipDeviceSynchronize();  // no kernel may still read the tables
    if (st->d_consts) (void)hipFree(st->d_consts);
    st->d_consts = nullptr;
    st->status = LSBM_ERR_NO_DEVICE;
    st->ready.store(false);
  }
  if (have_prev) (void)hipSetDevice(prev);
  return rc;
}

__attribute__((visibility("default"))) int lsbm_crc32c_fixed_dev(
    const void* d_base, uint64_t stride, uint64_t len, uint64_t n_blocks, const uint32_t* d_init,
    uint32_t* d_out, uint32_t flags, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_base || !d_out) return fail(LSBM_ERR_INVALID, "null pointer");
  if (flags & ~LSBM_CRC32C_MASKED) return fail(LSBM_ERR_INVALID, "unknown flags");
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  const uintptr_t b = reinterpret_cast<uintptr_t>(d_base);
  const bool fast = (b % 16 == 0) && (stride % 16 == 0) && len >= kRowBytes &&
                    (len % kRowBytes == 0) && stride >= len && stride <= (1ull << 28) &&
                    7 * stride + len < (1ull << 31) &&
                    n_blocks < (1ull << 34);
  if (fast) {
    const gf2::Mat an = gf2::byte_pow((int64_t)len);
    const uint32_t k_value = gf2::apply(an, 0xffffffffu) ^ 0xffffffffu;
    // A big batch goes as back-to-back launches of fixed_split_blocks() blocks
    // on the caller's stream (one launch over a 10M-block
    // shard ran 1-2 points under the same blocks a million at a time).
    const uint64_t per = fixed_split_blocks();
    hipStream_t hs = static_cast<hipStream_t>(stream);
    // the launches, and whether they take their groups from a cross-XCC queue:
    // one set of heads per launch, zeroed here, in stream-ordered scratch
    uint64_t launches = 0, min_m = n_blocks;
    for (uint64_t f = 0; f < n_blocks; launches++) {
      const uint64_t m = (per && n_blocks - f >= 2 * per) ? per : n_blocks - f;
      min_m = std::min(min_m, m);
      f += m;
    }
    uint32_t* heads = nullptr;
    const uint64_t nwaves = (uint64_t)st->num_cus * kWavesPerWg;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (fixed_queue_on() && (min_m + 7) / 8 >= 4 * nwaves && hipStreamIsCapturing(hs, &cap) == hipSuccess &&
        cap == hipStreamCaptureStatusNone) {
      const size_t bytes = launches * kQueueWords * sizeof(uint32_t);
      if (hipMallocAsync(reinterpret_cast<void**>(&heads), bytes, hs) != hipSuccess) {
        (void)hipGetLastError();
        heads = nullptr;
      } else if (hipMemsetAsync(heads, 0, bytes, hs) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFreeAsync(heads, hs);
        heads = nullptr;
      }
    }
    hipError_t e = hipSuccess;
    uint64_t li = 0;
    for (uint64_t f = 0; f < n_blocks && e == hipSuccess; li++) {
      const uint64_t m = (per && n_blocks - f >= 2 * per) ? per : n_blocks - f;
      e = launch_fixed(static_cast<const uint8_t*>(d_base) + f * stride, stride,
                       (uint32_t)(len / kRowBytes), m, d_init ? d_init + f : nullptr, d_out + f, flags,
                       k_value, st->d_consts, grid_for(st, m), hs, heads ? heads + li * kQueueWords : nullptr);
      f += m;
    }
    if (heads) (void)hipFreeAsync(heads, hs);
    return e == hipSuccess ? LSBM_OK : fail_hip(e, "crc32c_fixed_kernel");
  }
  // Any other geometry: the ragged kernel with fixed-stride extents.
  RaggedArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.stride = stride;
  a.len = len;
  a.extents = kExtFixed;
  a.n = n_blocks;
  a.init = d_init;
  a.out = d_out;
  a.flags = flags;
  a.mode = kModeOut;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_crc32c_batch_dev(
    const void* d_base, const uint64_t* d_offsets, uint64_t n_blocks, const uint32_t* d_init,
    uint32_t* d_out, uint32_t flags, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_base || !d_offsets || !d_out) return fail(LSBM_ERR_INVALID, "null pointer");
  if (flags & ~LSBM_CRC32C_MASKED) return fail(LSBM_ERR_INVALID, "unknown flags");
  RaggedArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.n = n_blocks;
  a.init = d_init;
  a.out = d_out;
  a.flags = flags;
  a.mode = kModeOut;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_crc32c_extents_dev(
    const void* d_base, const uint64_t* d_extents, uint64_t n_blocks, const uint32_t* d_init,
    uint32_t* d_out, uint32_t flags, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_base || !d_extents || !d_out) return fail(LSBM_ERR_INVALID, "null pointer");
  if (flags & ~LSBM_CRC32C_MASKED) return fail(LSBM_ERR_INVALID, "unknown flags");
  RaggedArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.handles = d_extents;  // {offset, size} pairs, the BlockHandle layout
  a.extents = kExtHandles;
  a.n = n_blocks;
  a.init = d_init;
  a.out = d_out;
  a.flags = flags;
  a.mode = kModeOut;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_crc32c_verify_dev(
    const void* d_base, const uint64_t* d_offsets, uint64_t n_blocks, const uint32_t* d_init,
    const uint32_t* d_expect, uint8_t* d_ok, uint32_t* d_nbad, uint32_t flags, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_base || !d_offsets || !d_expect || !d_ok) return fail(LSBM_ERR_INVALID, "null pointer");
  if (flags & ~LSBM_CRC32C_MASKED) return fail(LSBM_ERR_INVALID, "unknown flags");
  RaggedArgs a = {};
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.n = n_blocks;
  a.init = d_init;
  a.expect = d_expect;
  a.ok = d_ok;
  a.nbad = d_nbad;
  a.flags = flags;
  a.mode = kModeVerify;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

// lsbm_sst_seal_dev; in_place: one pass, trailers as plain byte stores
static int sst_seal_impl(uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles, const uint8_t* d_types,
             uint64_t n_blocks, uint32_t* d_nbad, void* stream, bool in_place) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_file || !d_handles || !d_types) return fail(LSBM_ERR_INVALID, "null pointer");
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  RaggedArgs a = {};
  a.base = d_file;
  a.handles = d_handles;
  a.extents = kExtHandles;
  a.types = d_types;
  a.n = n_blocks;
  a.nbad = d_nbad;
  a.limit = file_bytes;
  // The CRCs densely into stream-ordered scratch (the read-streaming units
  // kernel at full speed), then the trailers merged in by compare-and-swap,
  // per wave after its last row (trailer writes
  // interleaved with the reads cost 13 points).  Without scratch: in place,
  // one pass.
  // Small batches stay one pass: the scratch (and, in round 2, the second
  // launch) cost a fixed ~10 us, the deferred trailers save ~0.13 us per
  // block (config 1's 45K blocks: 0.088 ms one pass, 0.099 ms two; round 3's
  // per-wave merges: 0.092 one pass, 0.096 merged, profiles/r03/sealmin/).
  // Under hipGraph capture: one pass as well (no stream-ordered allocation
  // inside a captured sequence; an unknown capture state counts as capturing).
  uint32_t* crcs = nullptr;
  static const bool one_pass = getenv("LSBM_SEAL_ONE_PASS") != nullptr;  // (A/B measurements)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
  static const uint64_t min_blocks = [] {  // (A/B measurements)
    const char* e = getenv("LSBM_SEAL_MIN_BLOCKS");
    return e ? strtoull(e, nullptr, 10) : (1ull << 17);
  }();
  if (in_place || one_pass || capturing || n_blocks < min_blocks ||
      hipMallocAsync(reinterpret_cast<void**>(&crcs), n_blocks * sizeof(uint32_t), s) != hipSuccess) {
    (void)hipGetLastError();
    a.file = d_file;
    a.mode = kModeSstSeal;
    return run_ragged(a, s);
  }
  a.out = crcs;
  a.mode = kModeSstCrc;
  // Each wave merges its own blocks' trailers after its last row (the units
  // kernel's SstCrc epilogue, a.file set); LSBM_SEAL_SCATTER=1 keeps round 2's
  // separate compare-and-swap pass (A/B).
  static const bool scatter_pass = getenv("LSBM_SEAL_SCATTER") != nullptr;
  if (!scatter_pass) a.file = d_file;
  rc = run_ragged(a, s);
  if (rc == LSBM_OK && scatter_pass) {
    const hipError_t e = launch_trailer_scatter(d_file, file_bytes, d_handles, d_types, crcs, n_blocks,
                                                st->num_cus * 8, s);
    if (e != hipSuccess) rc = fail_hip(e, "trailer_scatter_kernel");
  }
  (void)hipFreeAsync(crcs, s);
  return rc;
}

__attribute__((visibility("default"))) int lsbm_sst_seal_dev(uint8_t* d_file, uint64_t file_bytes,
                                                             const uint64_t* d_handles,
                                                             const uint8_t* d_types,
                                                             uint64_t n_blocks, uint32_t* d_nbad,
                                                             void* stream) {
  return sst_seal_impl(d_file, file_bytes, d_handles, d_types, n_blocks, d_nbad, stream, false);
}

__attribute__((visibility("default"))) int lsbm_sst_trailer_crcs_dev(
    const uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles, const uint8_t* d_types,
    uint64_t n_blocks, uint32_t* d_masked, uint32_t* d_nbad, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_file || !d_handles || !d_types || !d_masked) return fail(LSBM_ERR_INVALID, "null pointer");
  RaggedArgs a = {};
  a.base = d_file;
  a.handles = d_handles;
  a.extents = kExtHandles;
  a.types = d_types;
  a.n = n_blocks;
  a.out = d_masked;
  a.nbad = d_nbad;
  a.limit = file_bytes;
  a.mode = kModeSstCrc;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_sst_verify_dev(const uint8_t* d_file,
                                                               uint64_t file_bytes,
                                                               const uint64_t* d_handles,
                                                               uint64_t n_blocks, uint8_t* d_ok,
                                                               uint32_t* d_nbad, void* stream) {
  if (n_blocks == 0) return LSBM_OK;
  if (!d_file || !d_handles || !d_ok) return fail(LSBM_ERR_INVALID, "null pointer");
  RaggedArgs a = {};
  a.base = d_file;
  a.handles = d_handles;
  a.extents = kExtHandles;
  a.limit = file_bytes;
  a.n = n_blocks;
  a.ok = d_ok;
  a.nbad = d_nbad;
  a.mode = kModeSstVerify;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_log_seal_dev(uint8_t* d_log, uint64_t log_bytes,
                                                             const uint64_t* d_headers,
                                                             uint64_t n_records,
                                                             uint32_t* d_masked, uint32_t* d_nbad,
                                                             void* stream) {
  if (n_records == 0) return LSBM_OK;
  if (!d_log || !d_headers) return fail(LSBM_ERR_INVALID, "null pointer");
  // One launch: WAL records are short (~1.2 KB), and a separate header pass
  // costs more than the in-kernel header writes do (A/B on 415K records:
  // 0.167 vs 0.155 ms, round 2).
  RaggedArgs a = {};
  a.base = d_log;
  a.file = d_log;
  a.handles = d_headers;
  a.extents = kExtLogHeaders;
  a.limit = log_bytes;
  a.n = n_records;
  a.out = d_masked;
  a.nbad = d_nbad;
  a.mode = kModeLogSeal;
  // Deferred headers (stream kernel): the masked CRCs densely into d_masked,
  // the header stores after each wave's last row -- 48.7-48.9% -> 49.6-49.7%
  // of HBM peak on 415K records (profiles/r03/logdefer/).  Without d_masked
  // the stores stay in place: stream-ordered scratch for the CRCs costs what
  // deferring saves (48.4-48.7% vs 48.6-48.8%).  LSBM_LOG_DEFER=0 / 1 turns
  // deferring off / on with scratch (A/B measurements).
  static const int defer_env = [] {
    const char* e = getenv("LSBM_LOG_DEFER");
    return e ? atoi(e) : -1;
  }();
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (defer_env == 0 || (defer_env < 0 && !d_masked)) return run_ragged(a, s);
  a.flags |= kFlagDeferHeaders;
  if (d_masked) return run_ragged(a, s);
  uint32_t* crcs = nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
  if (capturing || n_records < (1u << 17) ||
      hipMallocAsync(reinterpret_cast<void**>(&crcs), n_records * sizeof(uint32_t), s) != hipSuccess) {
    (void)hipGetLastError();
    a.flags &= ~kFlagDeferHeaders;
    return run_ragged(a, s);
  }
  a.out = crcs;
  const int rc = run_ragged(a, s);
  (void)hipFreeAsync(crcs, s);
  return rc;
}

__attribute__((visibility("default"))) int lsbm_log_crcs_dev(const uint8_t* d_log,
                                                             uint64_t log_bytes,
                                                             const uint64_t* d_headers,
                                                             uint64_t n_records,
                                                             uint32_t* d_masked, uint32_t* d_nbad,
                                                             void* stream) {
  if (n_records == 0) return LSBM_OK;
  if (!d_log || !d_headers || !d_masked) return fail(LSBM_ERR_INVALID, "null pointer");
  RaggedArgs a = {};
  a.base = d_log;
  a.file = nullptr;  // the image is not written
  a.handles = d_headers;
  a.extents = kExtLogHeaders;
  a.limit = log_bytes;
  a.n = n_records;
  a.out = d_masked;
  a.nbad = d_nbad;
  a.mode = kModeLogSeal;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_log_verify_dev(const uint8_t* d_log,
                                                               uint64_t log_bytes,
                                                               const uint64_t* d_headers,
                                                               uint64_t n_records, uint8_t* d_ok,
                                                               uint32_t* d_nbad, void* stream) {
  if (n_records == 0) return LSBM_OK;
  if (!d_log || !d_headers || !d_ok) return fail(LSBM_ERR_INVALID, "null pointer");
  RaggedArgs a = {};
  a.base = d_log;
  a.handles = d_headers;
  a.extents = kExtLogHeaders;
  a.limit = log_bytes;
  a.n = n_records;
  a.ok = d_ok;
  a.nbad = d_nbad;
  a.mode = kModeLogVerify;
  return run_ragged(a, static_cast<hipStream_t>(stream));
}

__attribute__((visibility("default"))) int lsbm_gather_dev(const void* d_src, const uint64_t* d_src_off,
                                                           const uint64_t* d_len, uint64_t n,
                                                           void* d_dst, const uint64_t* d_dst_off,
                                                           void* stream) {
  if (n == 0) return LSBM_OK;
  if (!d_src || !d_src_off || !d_len || !d_dst || !d_dst_off)
    return fail(LSBM_ERR_INVALID, "null pointer");
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  hipError_t e = launch_gather(static_cast<const uint8_t*>(d_src), d_src_off, d_len, n,
                               static_cast<uint8_t*>(d_dst), d_dst_off, st->num_cus * 8,
                               static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : fail_hip(e, "gather_kernel");
}

__attribute__((visibility("default"))) int lsbm_fill_splitmix64_dev(void* d_buf, uint64_t nbytes,
                                                                    uint64_t seed, void* stream) {
  if (nbytes == 0) return LSBM_OK;
  if (!d_buf || (reinterpret_cast<uintptr_t>(d_buf) & 15))
    return fail(LSBM_ERR_INVALID, "buffer must be 16-B aligned");
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  hipError_t e = launch_fill(static_cast<uint8_t*>(d_buf), nbytes, seed, st->num_cus * 8,
                             static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : fail_hip(e, "fill_splitmix64_kernel");
}

__attribute__((visibility("default"))) int lsbm_stream_read_dev(const void* d_buf, uint64_t nbytes,
                                                                uint32_t* d_sink, void* stream) {
  if (!d_buf || !d_sink || (reinterpret_cast<uintptr_t>(d_buf) & 15) || (nbytes & 15))
    return fail(LSBM_ERR_INVALID, "buffer must be 16-B aligned, nbytes % 16 == 0");
  DeviceState* st = nullptr;
  int rc = current_device(&st);
  if (rc != LSBM_OK) return rc;
  hipError_t e = launch_stream_read(d_buf, nbytes, d_sink, st->num_cus,
                                    static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LSBM_OK : fail_hip(e, "stream_read_kernel");
}

// The host-staged batch: chunks of whole blocks (<= 64 MiB, <= 64K blocks)
// through a leased HostSession's stages (host_session.h: per-device sessions,
// pinned staging on the device's NUMA node).  A chunk whose extents are in
// order and tight in page-locked memory is DMA-ed in place; any other chunk
// is gathered into the stage's pinned buffer by the worker pool, with its
// rebased offsets and init values behind the bytes (one DMA).  The kernel
// writes the CRCs straight into the stage's mapped host buffer.
__attribute__((visibility("default"))) int lsbm_crc32c_batch_host(int device, const void* h_base,
                                                                  const uint64_t* h_offsets,
                                                                  uint64_t n_blocks,
                                                                  const uint32_t* h_init,
                                                                  uint32_t* h_out,
                                                                  uint32_t flags) {
  if (n_blocks == 0) return LSBM_OK;
  if (!h_base || !h_offsets || !h_out) return fail(LSBM_ERR_INVALID, "null pointer");
  if (flags & ~LSBM_CRC32C_MASKED) return fail(LSBM_ERR_INVALID, "unknown flags");
  DeviceState* st = nullptr;
  int rc = ensure_device(device, &st);
  if (rc != LSBM_OK) return rc;
  SessionLease lease;
  {
    const Status os = lease.Open(device);
    if (!os.ok()) return fail(LSBM_ERR_HIP, os.ToString().c_str());
  }
  HostSession& hs = *lease;
  const uint8_t* src = static_cast<const uint8_t*>(h_base);
  const bool src_pinned = host_pinned(h_base, 1);  // (each chunk's range is checked before its DMA)
  // chunk size: LSBM_STAGE_CHUNK_MB overrides (tuning only; tools/host_sweep.py)
  static const uint64_t kChunkBytes = [] {
    const char* v = getenv("LSBM_STAGE_CHUNK_MB");
    const long mb = v ? atol(v) : 0;
    return (uint64_t)(mb > 0 && mb <= 1024 ? mb : 64) << 20;
  }();
  const uint64_t kChunkBlocks = kChunkBytes >> 10;
  const uint64_t meta_cap = (kChunkBlocks + 1) * 8 + kChunkBlocks * 4 + 512;
  struct Pending {
    uint64_t first = 0, count = 0;
  };
  Pending pend[HostSession::kStages];
  auto drain = [&](int i) -> int {
    Stage& s = hs.stage(i);
    if (!s.busy) return LSBM_OK;
    const hipError_t ee = hs.wait(s);
    if (ee != hipSuccess) return fail_hip(ee, "staged chunk");
    memcpy(h_out + pend[i].first, s.res.h, pend[i].count * 4);
    return LSBM_OK;
  };
  uint64_t next = 0;
  int si = 0;
  while (next < n_blocks && rc == LSBM_OK) {
    // the chunk [next, last)
    uint64_t bytes = 0, last = next;
    while (last < n_blocks && last - next < kChunkBlocks) {
      const uint64_t s0 = h_offsets[last], s1 = h_offsets[last + 1];
      const uint64_t len = s1 > s0 ? s1 - s0 : 0;
      if (last > next && bytes + len > kChunkBytes) break;
      bytes += len;
      last++;
    }
    const int i = si;
    si = (si + 1) % HostSession::kStages;
    Stage& s = hs.stage(i);
    if ((rc = drain(i)) != LSBM_OK) break;
    const uint64_t cnt = last - next;
    hipError_t e = s.bulk.reserve(std::max<uint64_t>(kChunkBytes, bytes) + meta_cap);
    if (e == hipSuccess) e = s.res.reserve_mapped(std::max<uint64_t>(kChunkBlocks, cnt) * 4);
    if (e != hipSuccess) {
      rc = fail_hip(e, "staging buffers");
      break;
    }
    // rebased offsets; a chunk whose extents are in order and tight can be
    // DMA-ed straight from a page-locked source, otherwise it is gathered
    bool tight = src_pinned;
    uint64_t pos = 0;
    for (uint64_t k = next; k < last && tight; k++) {
      const uint64_t s0 = h_offsets[k], s1 = h_offsets[k + 1];
      if (s0 != h_offsets[next] + pos) tight = false;
      pos += s1 > s0 ? s1 - s0 : 0;
    }
    if (tight && bytes) tight = host_pinned(src + h_offsets[next], bytes);
    // metadata behind the bytes (gathered) or at the buffer's start (tight)
    const uint64_t meta_off = tight ? 0 : (bytes + 15) / 16 * 16;
    uint64_t* off = reinterpret_cast<uint64_t*>(s.bulk.h + meta_off);
    pos = 0;
    for (uint64_t k = next; k < last; k++) {
      const uint64_t s0 = h_offsets[k], s1 = h_offsets[k + 1];
      off[k - next] = pos;
      pos += s1 > s0 ? s1 - s0 : 0;
    }
    off[cnt] = pos;
    uint32_t* ini = reinterpret_cast<uint32_t*>(off + cnt + 1);
    if (h_init) memcpy(ini, h_init + next, cnt * 4);
    const uint64_t meta_n = (cnt + 1) * 8 + (h_init ? cnt * 4 : 0);
    uint8_t* d_data = s.bulk.d + (tight ? (meta_n + 255) / 256 * 256 : 0);
    s.settled = false;  // (from here on the stage's stream may hold work)
    if (tight) {
      e = hipMemcpyAsync(s.bulk.d, s.bulk.h, meta_n, hipMemcpyHostToDevice, s.stream);
      if (e == hipSuccess && bytes)
        e = hipMemcpyAsync(d_data, src + h_offsets[next], bytes, hipMemcpyHostToDevice, s.stream);
    } else {
      // gather over the worker pool: runs of blocks of about equal bytes
      const int helpers = copy_helpers();
      const uint64_t ways = 2 * ((uint64_t)helpers + 1);
      const uint64_t per = std::max<uint64_t>(1, (cnt + ways - 1) / ways);
      parallel_for(
          bytes < (512u << 10) ? 1 : (size_t)((cnt + per - 1) / per),
          [&](size_t r) {
            const uint64_t k0 = next + r * per, k1 = std::min(last, k0 + per);
            for (uint64_t k = k0; k < k1; k++) {
              const uint64_t s0 = h_offsets[k], s1 = h_offsets[k + 1];
              if (s1 > s0) memcpy(s.bulk.h + off[k - next], src + s0, s1 - s0);
            }
          },
          helpers);
      e = hipMemcpyAsync(s.bulk.d, s.bulk.h, meta_off + meta_n, hipMemcpyHostToDevice, s.stream);
    }
    if (e != hipSuccess) {
      rc = fail_hip(e, "H2D");
      break;
    }
    uint8_t* d_meta = s.bulk.d + meta_off;
    RaggedArgs a = {};
    a.base = d_data;
    a.offsets = reinterpret_cast<const uint64_t*>(d_meta);
    a.n = cnt;
    a.init = h_init ? reinterpret_cast<const uint32_t*>(d_meta + (cnt + 1) * 8) : nullptr;
    a.out = reinterpret_cast<uint32_t*>(s.res.d);
    a.flags = flags;
    a.mode = kModeOut;
    a.dc = st->d_consts;
    a.u_noinit = u_noinit();
    e = launch_ragged(a, (int)st->num_cus, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) {
      rc = fail_hip(e, "staged launch");
      break;
    }
    s.busy = true;
    pend[i] = Pending{next, cnt};
    next = last;
  }
  for (int k = 0; k < HostSession::kStages; k++) {  // (any order: results go to their own slices)
    const int r2 = drain(k);
    if (rc == LSBM_OK) rc = r2;
  }
  return rc;
}

// Shards one host batch over several devices: contiguous runs of blocks of
// about equal bytes, one host thread per device, each bound to its device's
// NUMA node (its CPUs and its page placement, host_numa.h) and running the
// host-staged pipeline above on that device, whose staging sits on the same
// node.  No data moves between the devices (the CRCs are independent); each
// writes its slice of h_out.
__attribute__((visibility("default"))) int lsbm_crc32c_batch_host_multi(
    const int* devices, int n_devices, const void* h_base, const uint64_t* h_offsets,
    uint64_t n_blocks, const uint32_t* h_init, uint32_t* h_out, uint32_t flags) {
  if (n_blocks == 0) return LSBM_OK;
  if (!devices || n_devices <= 0 || !h_base || !h_offsets || !h_out)
    return fail(LSBM_ERR_INVALID, "null pointer or no devices");
  // shard boundaries by bytes (extents may be unsorted: fall back to counts)
  std::vector<uint64_t> cut(n_devices + 1, n_blocks);
  cut[0] = 0;
  uint64_t total = 0;
  bool sorted = true;
  for (uint64_t i = 0; i < n_blocks; i++) {
    const uint64_t s0 = h_offsets[i], s1 = h_offsets[i + 1];
    total += s1 > s0 ? s1 - s0 : 0;
    sorted = sorted && s1 >= s0;
  }
  if (sorted && total) {
    uint64_t acc = 0;
    int d = 1;
    for (uint64_t i = 0; i < n_blocks && d < n_devices; i++) {
      acc += h_offsets[i + 1] - h_offsets[i];
      while (d < n_devices && acc * n_devices >= total * (uint64_t)d) cut[d++] = i + 1;
    }
  } else {
    for (int d = 1; d < n_devices; d++) cut[d] = n_blocks * d / n_devices;
  }
  std::vector<int> rc(n_devices, LSBM_OK);
  std::vector<std::string> err(n_devices);
  std::vector<std::thread> th;
  for (int d = 0; d < n_devices; d++) {
    if (cut[d + 1] <= cut[d]) continue;
    th.emplace_back([&, d] {
      NumaBind nb(device_numa_node(devices[d]), true, true);
      const uint64_t lo = cut[d], cnt = cut[d + 1] - cut[d];
      rc[d] = lsbm_crc32c_batch_host(devices[d], h_base, h_offsets + lo, cnt,
                                     h_init ? h_init + lo : nullptr, h_out + lo, flags);
      if (rc[d] != LSBM_OK) err[d] = t_last_error;  // (per-thread error text)
    });
  }
  for (auto& t : th) t.join();
  for (int d = 0; d < n_devices; d++)
    if (rc[d] != LSBM_OK) return fail(rc[d], err[d].c_str());
  return LSBM_OK;
}

// Testing (include/lsbm_crc32c.h): the ragged kernel policy.
__attribute__((visibility("default"))) int lsbm_test_ragged_kernel(int which) {
  return set_ragged_policy(which) == 0 ? LSBM_OK : fail(LSBM_ERR_INVALID, "policy 0, 1 or 2");
}

}  // extern "C"

namespace lsbm {
int sst_seal_in_place(uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles, const uint8_t* d_types,
                      uint64_t n_blocks, hipStream_t stream) {
  return sst_seal_impl(d_file, file_bytes, d_handles, d_types, n_blocks, nullptr, stream, true);
}
}  // namespace lsbm
