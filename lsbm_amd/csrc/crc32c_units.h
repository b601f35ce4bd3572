// crc32c_units.h -- the ragged path's device code, shared by the units kernel
// (crc32c_kernels.hip) and the stream kernel (crc32c_stream.hip), which falls
// back to the units walk for a sub-piece whose extents are out of order.
//
// Both kernels compute, per block, exactly what lsbm's
// crc32c::Extend(init, block, n) returns (util/crc32c.cc:286-329).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace lsbm {

__shared__ uint32_t g_lds[kLdsWords];

// ---------------------------------------------------------------------------
// Cross-XCC work queue (round 6).  The eight XCDs of an MI355X do not read HBM
// at one rate: with every CU streaming, the waves of some XCDs (measured: the
// odd-numbered ones, 7% on average, 0-12% launch to launch) finish their
// share of a statically split batch tens of microseconds after the others,
// while within one XCD all workgroups end within ~10 us
// (tools/wave_spread_ragged.py).  No static split can
// know which XCD is slow, so past the first row the work is handed out at run
// time, in ITEMS of one group per wave of a workgroup:
//   * global: one head word per XCC (kQueueHeads, kQueueStride words apart),
//     head x hands out items 8 j + x, j = 0, 1, ... (every XCD streams the same
//     window of the batch), and a workgroup whose head is exhausted moves on
//     to the next head, so the fast XCDs take the slow ones' last items;
//   * per workgroup (WgQueue): the waves take slots k = 0, 1, ... from an LDS
//     counter; slot k is wave-group k % W of batch k / W, and batch b's item
//     is claimed from the heads by the wave that took slot 0 of batch b - 1
//     (kLead batches ahead) and published through an LDS ring of kRing
//     entries.  One global atomic per W groups, so the returning atomic --
//     ~5-7 us with every CU streaming, and retiring in order with the
//     claiming wave's row loads -- stalls one wave in W once per batch
//     (per-wave claims stalled every wave: 67-78% of HBM peak against 85%).
// Protocol (checked exhaustively-by-sampling in tests/test_queue_schedule.py):
// a workgroup's claims are made in batch order (publish(x) waits until batch
// x - 1 is published), so an exhausted queue (kNone) is seen in order and
// every claimed item is processed; entry x % kRing is reused only once all W
// readers of batch x - kRing have read it.  No wait can form a cycle (each
// waits only on smaller batches), and every spin is capped (kSpinCap): a
// protocol fault gives wrong results, which the tests see, never a hang.
// ---------------------------------------------------------------------------
// (kQueueHeads, kQueueStride, kQueueWords: crc32c_types.h)

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x & (kQueueHeads - 1);
}

// One claim from head h by lane 0; wave-uniform result.
__device__ __forceinline__ uint32_t queue_take(uint32_t* heads, uint32_t h) {
  uint32_t j = 0;
  if ((threadIdx.x & 63u) == 0) j = atomicAdd(heads + h * kQueueStride, 1u);
  return __builtin_amdgcn_readfirstlane(j);
}

constexpr uint32_t kWqRing = 4, kWqLead = 1, kWqNone = 0xffffffffu, kSpinCap = 1u << 20;
constexpr uint32_t kWqWords = 3 + 3 * kWqRing;  // next, head, exhausted, tag[R], item[R], read[R]
static_assert(kWqLead == 1, "wave 0 publishes batch 1 only: the batches before the first slot-0 taker's");
static_assert(kWqRing > kWqLead, "an entry is reused only after its batch's slots were all taken");

// LDS words by address space: a generic (flat) pointer would make every
// access a flat op, counted in vmcnt with the row loads (a spin would then
// wait for all of them)
typedef __attribute__((address_space(3))) uint32_t lds_u32;

template <uint32_t W>
struct WgQueue {
  uint32_t* heads;  // global heads
  lds_u32* s;       // LDS words (kWqWords)
  uint64_t items;   // items the heads hand out

  __device__ __forceinline__ volatile lds_u32* v(uint32_t i) const { return (volatile lds_u32*)(s + i); }
  // (thread 0, before a workgroup barrier)
  __device__ __forceinline__ void init(uint32_t xcc) const {
    *v(0) = W;  // slots 0 .. W-1: row 0, the waves' own
    *v(1) = xcc;
    *v(2) = 0;
    for (uint32_t e = 0; e < kWqRing; e++) {
      *v(3 + e) = 0;  // (tag 0: batch 0, which is never read)
      *v(3 + kWqRing + e) = kWqNone;
      *v(3 + 2 * kWqRing + e) = 0;
    }
  }
  __device__ __forceinline__ uint32_t take() const {
    uint32_t k = 0;
    if ((threadIdx.x & 63u) == 0) k = __atomic_fetch_add(s, 1u, __ATOMIC_RELAXED);
    return __builtin_amdgcn_readfirstlane(k);
  }
  __device__ __forceinline__ uint32_t rd(uint32_t i) const { return __builtin_amdgcn_readfirstlane(*v(i)); }
  // Claim batch x's item from the heads and publish it (wave-uniform).
  __device__ __forceinline__ void publish(uint32_t x) const {
    const uint32_t e = x % kWqRing, pe = (x - 1) % kWqRing;
    uint32_t spins = 0;
    if (x >= 2)  // in batch order
      while (rd(3 + pe) != x - 1 && ++spins < kSpinCap) __builtin_amdgcn_s_sleep(2);
    if (x > kWqRing)  // the entry's previous batch read by all W
      while (rd(3 + 2 * kWqRing + e) != W && ++spins < kSpinCap) __builtin_amdgcn_s_sleep(2);
    uint32_t h = rd(1), out = rd(2), it = kWqNone;
    while (spins < kSpinCap && out < kQueueHeads) {
      const uint64_t cand = (uint64_t)queue_take(heads, h) * kQueueHeads + h;
      if (cand < items) {
        it = (uint32_t)cand;
        break;
      }
      if (++out < kQueueHeads) h = (h + 1) & (kQueueHeads - 1);
    }
    if ((threadIdx.x & 63u) == 0) {  // (LDS ops of one wave complete in order: item before tag)
      *v(1) = h;
      *v(2) = out;
      *v(3 + kWqRing + e) = it;
      *v(3 + 2 * kWqRing + e) = 0;
      *v(3 + e) = x;
    }
  }
  // Batch b's item (kWqNone: the queue is exhausted), counted as read.
  __device__ __forceinline__ uint32_t read(uint32_t b) const {
    const uint32_t e = b % kWqRing;
    uint32_t spins = 0;
    while (rd(3 + e) != b)
      if (++spins >= kSpinCap) return kWqNone;
      else __builtin_amdgcn_s_sleep(2);
    const uint32_t it = rd(3 + kWqRing + e);
    if ((threadIdx.x & 63u) == 0) __atomic_fetch_add(s + 3 + 2 * kWqRing + e, 1u, __ATOMIC_RELAXED);
    return it;
  }
};

// Diagnostic builds only (-DLSBM_DIAG_STAMPS, tools/wave_spread.py): every
// wave stamps its start (0), its first data (1) and its end (2) with
// s_memrealtime (100 MHz), and its XCC (3).  One array per kernel source
// (internal linkage), read by that source's lsbm_diag_stamps* export.
#ifdef LSBM_DIAG_STAMPS
static __device__ uint64_t g_stamps[4][65536];
#define DIAG_STAMP_W(k, w)                                                          \
  do {                                                                              \
    if ((threadIdx.x & 63u) == 0) g_stamps[k][(w) & 65535] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define DIAG_XCC_W(w)                                                               \
  do {                                                                              \
    if ((threadIdx.x & 63u) == 0) {                                                 \
      uint32_t xcc_;                                                                \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_));     \
      g_stamps[3][(w) & 65535] = xcc_;                                              \
    }                                                                               \
  } while (0)
#else
#define DIAG_STAMP_W(k, w) do { } while (0)
#define DIAG_XCC_W(w) do { } while (0)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Global-address-space pointer: addresses built from integers would otherwise
// be generic (flat) loads, which count on lgkmcnt too and force full drains.
typedef const __attribute__((address_space(1))) u32x4* gptr_u32x4;

#ifndef LSBM_UNIT_ROWS  // longest unit of general ragged batches (ablation builds override)
#define LSBM_UNIT_ROWS kUnitRows
#endif

// c_m = A^128(c_m) ^ w_m for the four braids of one 16-B row slice.
#define STEP_ROW(W)                                           \
  do {                                                        \
    c0 = row_step(g_lds, c0, (W).x, L0, L1, L2, L3);          \
    c1 = row_step(g_lds, c1, (W).y, L0, L1, L2, L3);          \
    c2 = row_step(g_lds, c2, (W).z, L0, L1, L2, L3);          \
    c3 = row_step(g_lds, c3, (W).w, L0, L1, L2, L3);          \
  } while (0)

// ---------------------------------------------------------------------------
// Ragged path: one kernel, every output mode.
//
// Frame.  Rows are 128-B aligned in the absolute address space, so every load
// is an aligned 16-B load whatever the block's alignment.  For block [s, e):
//   * bytes of the frame outside [s, e) are zero; leading zeros leave a raw
//     CRC unchanged, so the frame may start early for free;
//   * the init register v = init ^ ~0 is injected as 4 virtual bytes
//     u = A^-4(v) at [s-4, s) (absorbing u from zero gives exactly v);
//   * the frame ends z = frame_end - e bytes late: undone with A^-z.
// Units.  The frame is cut into units of <= kMaxRows rows (crc32c_types.h).
// Each wave walks a contiguous range of blocks and hands the next 8 units of
// the range to its 8 lane groups.  A unit's raw CRC, shifted to the frame end
// by A^(128 k), is summed with the other units of its block INSIDE the wave:
// the units of a round are consecutive, so a segmented xor-scan over the 8
// groups sums each block's units of the round, and the one block that is still
// open at the end of a round carries its partial sum into the next round.  The
// group holding a block's last unit finishes it in registers (A^-z, the mode:
// CRC, verify, SSTable trailer, log header), so there is no accumulator array,
// no atomics on the data path and no second kernel.
// ---------------------------------------------------------------------------
// Byte n of a little-endian word and below: (1 << 8n) - 1, n in [0, 4].
__device__ __forceinline__ uint32_t low_bytes(int32_t n) {
  return (uint32_t)((1ull << (8 * n)) - 1ull);
}

// The word at byte p of a 16-B chunk, fixed for the frame: keep the bytes in
// [ds, de) (s and e relative to the chunk) and add the virtual init bytes u
// at [ds - 4, ds).
__device__ __forceinline__ uint32_t fix_word(uint32_t w, int32_t ds, int32_t de, uint32_t u,
                                             int32_t p) {
  const int32_t lo = min(max(ds - p, 0), 4), hi = min(max(de - p, 0), 4);
  const uint32_t keep = low_bytes(hi) & ~low_bytes(lo);
  const int32_t d = p + 4 - ds;  // the word's offset from s - 4
  uint32_t inj = 0;
  if (d >= 0 && d < 4) inj = u >> (8 * d);
  else if (d < 0 && d > -4) inj = u << (-8 * d);
  return (w & keep) ^ inj;
}

// The two 64-bit words that define block b's extent (offsets[b], offsets[b+1]
// or a BlockHandle {offset, size}); nothing is loaded for fixed extents.
struct ExtRaw {
  uint64_t x, y;
};
typedef const __attribute__((address_space(1))) uint64_t* gptr_u64;
typedef const __attribute__((address_space(1))) uint32_t* gptr_u32;
typedef const __attribute__((address_space(1))) uint8_t* gptr_u8;

constexpr uint64_t kLogHeaderSize = 7;  // common/log_format.h:30 (crc 4, length 2, type 1)
constexpr uint64_t kLogNoHeader = ~0ull;  // ExtRaw.y of a header that is not inside the image
constexpr uint64_t kTrailer = 5;        // table/format.h:84 kBlockTrailerSize

// Log headers: this loads the header offset only (r.x); log_length() adds the
// record length, a load that depends on it (see crc32c_units_kernel).
__device__ __forceinline__ ExtRaw load_ext_raw(const RaggedArgs& a, uint64_t b) {
  ExtRaw r = {0, 0};
  if (a.extents == kExtLogHeaders) {
    const gptr_u64 h = reinterpret_cast<gptr_u64>(reinterpret_cast<uint64_t>(a.handles));
    r.x = h[b];
  } else if (a.extents == kExtHandles) {
    const gptr_u64 h = reinterpret_cast<gptr_u64>(reinterpret_cast<uint64_t>(a.handles));
    r.x = h[2 * b];
    r.y = h[2 * b + 1];
  } else if (a.extents == kExtOffsets) {
    const gptr_u64 o = reinterpret_cast<gptr_u64>(reinterpret_cast<uint64_t>(a.offsets));
    r.x = o[b];
    r.y = o[b + 1];
  }
  return r;
}

// The record length (LE16 at header + 4, read byte-wise) into r.y; a header
// that does not fit the image reads the zero pad instead and gets kLogNoHeader.
__device__ __forceinline__ void log_length(const RaggedArgs& a, ExtRaw& r) {
  const bool inside = r.x <= a.limit && a.limit - r.x >= kLogHeaderSize;
  uint64_t p = inside ? reinterpret_cast<uint64_t>(a.base) + r.x + 4
                      : reinterpret_cast<uint64_t>(a.dc->zero16);
  asm volatile("" : "+v"(p));  // defined in every lane (see crc32c_units_kernel)
  const gptr_u8 q = reinterpret_cast<gptr_u8>(p);
  const uint64_t len = (uint64_t)q[0] | ((uint64_t)q[1] << 8);
  r.y = inside ? len : kLogNoHeader;
}

// Block b's extent [s, e) as absolute addresses, whether the record fits the
// image (log headers; SSTable handles whose n + 5 bytes must lie inside
// `limit`, table/format.cc:88-91), and the address of its stored / written
// checksum: the trailer's type byte (seal: e), the trailer's crc (verify: e,
// the extent covers the type byte), the log header (log modes).  A record
// that does not fit is empty here (no byte of it is read) and bad at finish.
__device__ __forceinline__ void extent_from_raw(const RaggedArgs& a, uint64_t b, ExtRaw r,
                                                uint64_t& s, uint64_t& e, bool& fits,
                                                uint64_t& at) {
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  fits = true;
  if (a.extents == kExtLogHeaders) {
    // CRC over [type || payload] = [h + 6, h + 7 + length) (common/log_reader.cc:231)
    fits = r.y != kLogNoHeader && a.limit - r.x - kLogHeaderSize >= r.y;
    s = base + (fits ? r.x + 6 : 0);
    e = fits ? s + 1 + r.y : s;
    at = base + r.x;
  } else if (a.extents == kExtHandles) {
    if (a.mode == kModeSstSeal || a.mode == kModeSstVerify || a.mode == kModeSstCrc)
      fits = r.x <= a.limit && a.limit - r.x >= kTrailer && a.limit - r.x - kTrailer >= r.y;
    s = base + (fits ? r.x : 0);
    e = fits ? s + r.y + (a.mode == kModeSstVerify ? 1u : 0u) : s;  // verify covers the type
    at = e;
  } else if (a.extents == kExtFixed) {
    s = base + b * a.stride;
    e = s + a.len;
    at = e;
  } else {
    s = base + r.x;
    e = base + r.y;
    if (e < s) e = s;
    at = e;
  }
}

// a / b for b >= 1: float reciprocal and one correction each way (exact for
// a < 2^24, i.e. blocks under 2 GiB); the integer divide beyond that.
__device__ __forceinline__ uint32_t div_u32(uint32_t a, uint32_t b) {
  if (a >= (1u << 24)) return a / b;
  uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
  const int32_t r = (int32_t)(a - q * b);
  q = r < 0 ? q - 1u : ((uint32_t)r >= b ? q + 1u : q);
  return q;
}

struct Frame {
  uint64_t s, e, row0, rows;  // rows >= 1
  uint32_t units;             // ceil(rows / max_rows)
  uint32_t q, rem;            // balanced split: units of q rows, the first rem of them q + 1
};

__device__ __forceinline__ Frame frame_of(uint64_t s, uint64_t e, uint32_t max_rows) {
  Frame f;
  f.s = s;
  f.e = e;
  f.row0 = (s - 4) >> 7;
  const uint64_t row_end = (e + 127) >> 7;
  f.rows = row_end > f.row0 ? row_end - f.row0 : 1;
  // rows < 2^32 (blocks under 512 GiB): 32-bit unit arithmetic
  const uint32_t r32 = (uint32_t)f.rows;
  f.units = (r32 + max_rows - 1) / max_rows;  // constant divisor: multiply-high
  f.q = f.units == 1u ? r32 : div_u32(r32, f.units);
  f.rem = r32 - f.q * f.units;
  return f;
}

// M(v) for nibble tables in LDS at byte offset `tab` (low 6 bits clear).
__device__ __forceinline__ uint32_t nib_lds_at(const uint32_t* lds, uint32_t tab, uint32_t v) {
  uint32_t t[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t f = q == 0 ? (v << 2) : (v >> (4 * q - 2));
    t[q] = lds_load(lds, ((f & 0x3cu) | tab) + q * 64);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// A^(128 k)(v), k rows, k a multiple of 2^kRowPowLo (the column tables take
// the low bits): LDS tables for bits kRowPowLo..kRowPowTables-1 of k, global
// ones beyond.
__device__ __forceinline__ uint32_t shift_rows(const uint32_t* lds, const DevConsts* dc,
                                               uint32_t v, uint64_t k) {
  static_assert(kShiftCols == 1u << kRowPowLo, "column shifts cover the low bits");
  k >>= kRowPowLo;
  for (uint32_t i = kRowPowLo; k; i++, k >>= 1)
    if (k & 1u)
      v = i < kRowPowTables ? nib_lds_at(lds, kNibRowPow + i * 512, v) : nib_glb(dc->pow_nib[7 + i], v);
  return v;
}

// M(v) for a matrix in column form spread over an 8-lane group: lane li holds
// columns 4li .. 4li+3 (M(1 << b) for the bits b of v in [4li, 4li + 4)).
// Every lane of the group receives M(v); every lane must execute it.
__device__ __forceinline__ uint32_t cols_apply(u32x4 c, uint32_t v, uint32_t li) {
  const uint32_t nib = v >> (4u * li);
  const uint32_t r = xor3(c.x & (0u - (nib & 1u)), c.y & (0u - ((nib >> 1) & 1u)),
                          c.z & (0u - ((nib >> 2) & 1u))) ^
                     (c.w & (0u - ((nib >> 3) & 1u)));
  return group_xor(r);
}

// A(t) for one byte t: the CRC register contribution of extending by a byte
// (util/crc32c.cc:291-294 with l = 0), computed bitwise.
__device__ __forceinline__ uint32_t advance_byte(uint32_t t) {
#pragma unroll
  for (int i = 0; i < 8; i++) t = (t >> 1) ^ (0x82F63B78u & (0u - (t & 1u)));
  return t;
}

// 4 bytes at an arbitrary address from the two aligned dwords covering them.
__device__ __forceinline__ uint32_t unaligned_word(uint32_t lo, uint32_t hi, uint64_t addr) {
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)addr & 3u);
}

// Start offset of block b in [0, n]: offsets[b]; a handle's offset, and the
// end of the last block for b = n.  Monotone for a sorted batch.
template <uint32_t kExt>
__device__ __forceinline__ uint64_t start_key(const RaggedArgs& a, uint64_t b) {
  if constexpr (kExt == kExtOffsets) {
    return reinterpret_cast<gptr_u64>(reinterpret_cast<uint64_t>(a.offsets))[b];
  } else {
    const gptr_u64 h = reinterpret_cast<gptr_u64>(reinterpret_cast<uint64_t>(a.handles));
    const uint64_t i = b < a.n ? b : a.n - 1;
    const uint64_t x = h[2 * i];
    return b < a.n ? x : x + h[2 * i + 1];
  }
}

// Byte-balanced ranges.  With block lengths drawn from a skewed distribution,
// equal block COUNTS per wave leave the heaviest wave ~9% above the mean (10M
// Zipf blocks over 4,096 waves), and the kernel waits for it.  The batch is
// cut into P pieces (one per wave, or one per wave and chunk); piece w is
// [f(w), f(w + 1)) with f(w) the first block whose start is at or past
// key(0) + (key(n) - key(0)) w / P.  Both ends are found together, lanes 0-31
// for f(w) and 32-63 for f(w + 1), by a 32-ary search (one load per lane per
// step, ~5 steps for 10M blocks).  The search only ever compares key(p) >= t,
// so its result is non-decreasing in t for ANY key array: the pieces tile
// [0, n) exactly even for an unsorted batch (which is then merely not
// balanced).  P < 2^32.
template <uint32_t kExt>
__device__ __forceinline__ void byte_ranges(const RaggedArgs& a, uint64_t wave, uint64_t P,
                                            uint64_t& b_lo, uint64_t& b_hi) {
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, k = lane & 31u;
  const uint64_t k0 = start_key<kExt>(a, 0), kn = start_key<kExt>(a, a.n);
  if (kn <= k0) return;  // (wave-uniform) keep the equal counts
  const uint64_t w = wave + half;
  const uint64_t D = kn - k0;
  const uint64_t t = k0 + (D / P) * w + ((D % P) * w) / P;  // k0 + floor(D w / P), no overflow
  // the answer lies in [lo, hi]; hi when no key in [lo, hi) reaches t.
  // f(0) = 0 and f(P) = n.
  uint64_t lo = w >= P ? a.n : 0, hi = w == 0 ? 0 : a.n;
  for (;;) {
    if (__ballot(hi - lo > 32u) == 0ull) break;
    const uint64_t step = (hi - lo + 31u) >> 5;
    uint64_t p = lo + (k + 1) * step - 1u;
    p = hi > lo ? (p < hi ? p : hi - 1u) : 0u;  // every load in [0, n]
    const bool ge = hi > lo && start_key<kExt>(a, p) >= t;
    const uint32_t m = (uint32_t)(__ballot(ge) >> (32u * half));
    if (hi - lo > 32u) {
      if (m == 0u) {
        lo = hi;
      } else {
        const uint32_t ks = (uint32_t)__builtin_ctz(m);
        const uint64_t pk = (uint64_t)__shfl((unsigned long long)p, (int)(32u * half + ks));
        lo = lo + ks * step;
        hi = pk;
      }
    }
  }
  const uint64_t q = lo + k < hi ? lo + k : 0u;
  const bool ge = lo + k < hi && start_key<kExt>(a, q) >= t;
  const uint32_t m = (uint32_t)(__ballot(ge) >> (32u * half));
  const uint64_t f = m ? lo + (uint32_t)__builtin_ctz(m) : hi;
  auto read64 = [](uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
  };
  b_lo = read64(f, 0);
  b_hi = read64(f, 32);
}

// The chunked sweep's ranges: bounds[i] = f(i) for i in [0, P] (byte_ranges
// with P pieces; 32-bit, the sweep is for n < 2^32 - 1), one wave per two.
template <uint32_t kExt>
__global__ __launch_bounds__(256) void range_bounds_kernel(RaggedArgs args, uint64_t P, uint32_t* bounds) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = (uint64_t)gridDim.x * 4u;
  for (uint64_t q = (uint64_t)blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
       2 * q <= P; q += nw) {
    uint64_t lo = args.n * (2 * q) / P, hi = 2 * q + 1 <= P ? args.n * (2 * q + 1) / P : args.n;
    byte_ranges<kExt>(args, 2 * q, P, lo, hi);
    if (lane == 0) bounds[2 * q] = (uint32_t)lo;  // (n < 2^32 - 1 here)
    if (lane == 32 && 2 * q + 1 <= P) bounds[2 * q + 1] = (uint32_t)hi;
  }
}

// Units kernel.  Each wave owns a contiguous range of blocks and walks it in
// rounds of 8 units (one per lane group).  The loop is software-pipelined so
// that no global-memory latency is exposed between rounds:
//   * the extents of the next round's blocks are loaded one round ahead;
//   * a round loads what its units' finish will need (shift and A^-z
//     matrices, expected values, stored trailers) before its row loads, and
//     consumes them one round later, so no wait ever drains the row loads;
//   * a round issues its first bank of row loads, THEN retires the previous
//     round (merge, shift, in-wave sum, finish: LDS and ALU work overlapping
//     the loads), then streams its rows.
//
// kMaxRows is the longest unit: kUnitRows for general batches; kSstUnitRows for
// SSTable trailers, whose blocks (4,117-4,123 B with the type byte, 33-34 rows)
// then go through as ONE unit each, 8 blocks per round, no split and no shift.
// This wave's first range of blocks.  Big general batches are swept in
// chunks (args.bounds, from range_bounds_kernel): the batch is cut into
// nchunks chunks of about kChunkBlocks * nwaves blocks, each chunk into nwaves
// byte-balanced ranges, and wave w walks its range of every chunk in turn, so
// that all waves move through the batch together, one chunk at a time (128
// blocks per wave: 6.5 GB of config 4's blocks; A/B 32 / 64 / 128 / 256
// blocks, profiles/r02/ab/s62_s63_sweep_chunks.log: 128 and 256 best, +1.5-2
// points on config 4, +2-3 on 117 GiB of equal 12 KiB blocks).
// With one contiguous range per wave, the waves' streams spread over the
// whole batch and the rate fell with its size: 81% of HBM peak for 16 GiB
// of equal 12 KiB blocks, 78% for 64 GiB, 75% for 117 GiB, and 78% for the
// 117 GiB as 7 separate launches (profiles/r02/ab/s58_usweep_size.log,
// s61_size_effect.log).  Range ends are block ends, so no block's units
// straddle two ranges.  (n < 2^32 - 1 there: round keys are 32-bit block
// indices relative to the wave's first block.)  Other batches: one range
// per wave, equal counts, or equal bytes for general batches (whose lengths
// may be skewed; SSTable blocks and log records are near-uniform).
// chunked: piece index pi = c * nwaves + w of the range being walked, and
// p_end the end of the pieces (nchunks * nwaves < 2^32); the chunked walk
// reads its ranges from args.bounds itself (b_lo / b_hi unset).
// SSTable modes over a handle batch: equal-count pieces (piece_range), no
// bounds table -- their blocks are near-uniform (one unit each).
template <uint32_t kMode, uint32_t kExt>
constexpr bool kArithPieces = (kMode == kModeSstVerify || kMode == kModeSstCrc) && kExt == kExtHandles;
// modes whose batches can be swept in pieces (chunked)
template <uint32_t kMode, uint32_t kExt>
constexpr bool kCanChunk = ((kMode == kModeOut || kMode == kModeVerify) && (kExt == kExtOffsets || kExt == kExtHandles)) ||
                           kArithPieces<kMode, kExt>;

template <uint32_t kMode, uint32_t kExt>
__device__ __forceinline__ void wave_range(const RaggedArgs& args, uint64_t wave, uint64_t nwaves,
                                           bool& chunked, uint32_t& pi, uint32_t& p_end,
                                           uint64_t& b_lo, uint64_t& b_hi) {
  constexpr bool kChunkable = (kMode == kModeOut || kMode == kModeVerify) &&
                              (kExt == kExtOffsets || kExt == kExtHandles);
  chunked = (kChunkable && args.bounds != nullptr) || (kArithPieces<kMode, kExt> && args.nchunks != 0);
  pi = (uint32_t)wave;
  p_end = (uint32_t)(args.nchunks * nwaves);
  b_lo = args.n * wave / nwaves;
  b_hi = args.n * (wave + 1) / nwaves;
  if (!chunked) {
#ifndef LSBM_NO_BALANCE  // A/B builds only
    // (log records too by bytes, keyed on header offsets: 3 points slower on a
    // 0.5 GB WAL, the search's latency costs more than the uneven counts;
    // profiles/r02/ab/s56_log_byte_ranges.log)
    if constexpr ((kMode == kModeOut || kMode == kModeVerify) &&
                  (kExt == kExtOffsets || kExt == kExtHandles))
      if (args.n >= 16u * nwaves) byte_ranges<kExt>(args, wave, nwaves, b_lo, b_hi);
#endif
  }
}

// Piece i of a chunked sweep: [bounds[i], bounds[i + 1]) from the bounds
// table, or, without one (kArithPieces), the equal-count cut of the batch
// into P = nchunks * nwaves pieces (RaggedArgs piece_q, piece_r).
__device__ __forceinline__ void piece_range(const RaggedArgs& a, uint32_t i, uint32_t P, uint64_t& lo,
                                            uint64_t& hi) {
  if (a.bounds) {
    lo = a.bounds[i];
    hi = a.bounds[i + 1];
  } else {
    (void)P;
    lo = (uint64_t)i * a.piece_q + (i < a.piece_r ? i : a.piece_r);
    hi = lo + a.piece_q + (i < a.piece_r ? 1u : 0u);
  }
}

// Which piece a wave walks next.  Static (LSBM_PIECES_STATIC, A/B): its own
// range of the next chunk, pi + nwaves.  Default (round 6): the workgroup's
// waves take their pieces in turn from an LDS counter -- the fixed kernel's
// round-5 schedule -- so a fast wave takes more of them: slot k of the
// workgroup is piece (k / W) nwaves + W blockIdx + k % W (the static sweep's
// pieces of this workgroup; each wave's first piece is its own, k = W is the
// first claim).  (On units and stream kernels the static split left the
// waves of one workgroup ending up to ~100 us apart on a 0.65 ms launch:
// tools/wave_spread_ragged.py)
template <uint32_t W>
__device__ __forceinline__ uint32_t next_piece(lds_u32* claim, uint32_t pi, uint64_t nwaves) {
#ifndef LSBM_PIECES_STATIC
  if (claim) {
    uint32_t k = 0;
    if ((threadIdx.x & 63u) == 0) k = __atomic_fetch_add(claim, 1u, __ATOMIC_RELAXED);
    k = __builtin_amdgcn_readfirstlane(k);
    return (k / W) * (uint32_t)nwaves + blockIdx.x * W + k % W;
  }
#endif
  return pi + (uint32_t)nwaves;
}

// Rows of a round the walk absorbs at raised wave priority (units_walk;
// 8, 12, 16, ...: the row loop's bank boundaries).
#ifndef LSBM_PRIO_ROWS  // (A/B builds override)
#define LSBM_PRIO_ROWS 16
#endif
constexpr uint32_t kPrioRows = LSBM_PRIO_ROWS;
static_assert(kPrioRows >= 8 && kPrioRows % 4 == 0, "priority lowered at a bank boundary of the row loop");

// The units walk: the blocks [b_lo, b_hi) (or, chunked, this wave's range of
// every chunk) in rounds of 8 units.  crc32c_units_kernel runs it over the
// wave's range; crc32c_stream_kernel runs it over a sub-piece whose extents
// are not in order (load_tables false: the LDS tables are in place).
//
// first_lo: the walk starts at block first_lo (>= the range's start) of its
// first range; the stream kernel resumes there after streaming the blocks
// before it (chunked too: later ranges are walked whole).
// kClaim: the walk's pieces are claimed (claim, next_piece) -- a compile-time
// switch, so that the walks that never claim keep their registers; kChunks
// false: a walk of one range (chunked_in is false), compiled without the
// piece code (the SSTable walks run at 128 VGPRs: the dead piece state cost
// their one-range walks, the fused seal's, 1.3 points).
template <uint32_t kMaxRows, uint32_t kMode, uint32_t kExt, bool kClaim = false, uint32_t kW = kWavesPerWg,
          bool kChunks = true>
__device__ __forceinline__ void units_walk(RaggedArgs args, const uint64_t wave, const uint64_t nwaves,
                                           uint64_t b_lo, uint64_t b_hi, const bool chunked_in,
                                           uint32_t pi, const uint32_t p_end, const bool load_tables,
                                           const uint64_t first_lo = 0, lds_u32* claim_arg = nullptr) {
  const bool chunked = kChunks && chunked_in;
  lds_u32* const claim = kClaim ? claim_arg : nullptr;
  args.mode = kMode;   // compile-time: lets the compiler drop the other modes' code
  args.extents = kExt;
  const DevConsts* __restrict__ dc = args.dc;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = row_lane_base(lane);
  const uint32_t L0 = lb | kRowTab[0], L1 = lb | kRowTab[1], L2 = lb | kRowTab[2], L3 = lb | kRowTab[3];
  const uint32_t lane_fin = kNibFin | lb;
  // Static pieces: the next chunk's range is loaded a chunk ahead (pf_*).
  // Claimed pieces (claim != null): the next piece is claimed when this one
  // ends -- a claim made ahead would hold the wave to it -- and its bounds
  // loaded then (equal-count pieces need no load).
  uint32_t pf_lo = 0, pf_hi = 0;
  bool pf = false;  // pf_* hold piece pi + nwaves
  auto piece = [&](uint32_t i, uint64_t& lo, uint64_t& hi) { piece_range(args, i, p_end, lo, hi); };
  // the next non-empty piece after pi into (pi, lo, hi); false: none left
  auto advance = [&](uint64_t& lo, uint64_t& hi) -> bool {
    for (;;) {
      const uint32_t np = claim ? next_piece<kW>(claim, pi, nwaves) : pi + (uint32_t)nwaves;
      if (np >= p_end) return false;
      if (!claim && pf && np == pi + (uint32_t)nwaves) {
        lo = pf_lo;
        hi = pf_hi;
      } else {
        piece(np, lo, hi);
      }
      pi = np;
      pf = false;
      if (lo < hi) break;
    }
#ifndef LSBM_NO_BOUNDS_PREFETCH  // A/B builds only
    if (!claim && pi + nwaves < p_end) {
      uint64_t l2, h2;
      piece(pi + (uint32_t)nwaves, l2, h2);
      pf_lo = (uint32_t)l2;
      pf_hi = (uint32_t)h2;
      pf = true;
    }
#endif
    return true;
  };
  if (chunked) {
    piece(pi, b_lo, b_hi);
    b_lo = b_lo < first_lo ? first_lo : b_lo;
    if (b_lo >= b_hi) {
      if (!advance(b_lo, b_hi)) b_lo = b_hi;  // (nothing left: an empty walk)
    } else {
#ifndef LSBM_NO_BOUNDS_PREFETCH
      if (!claim && pi + nwaves < p_end) {
        uint64_t l2, h2;
        piece(pi + (uint32_t)nwaves, l2, h2);
        pf_lo = (uint32_t)l2;
        pf_hi = (uint32_t)h2;
        pf = true;
      }
#endif
    }
  }
  const uint64_t dummy = reinterpret_cast<uint64_t>(dc->zero16);
  const uint32_t* __restrict__ init = args.init;
  constexpr uint32_t mode = kMode;
  const uint32_t jl = lane < 8u ? lane : 8u;  // lanes 0..8 hold the walk's 9 blocks
  // extents (+ init) of blocks nb + jl, clamped into the batch so that the
  // loads are unconditional; only lanes with nb + lane < range_hi walk them
  auto prefetch = [&](uint64_t nb, ExtRaw& r, uint32_t& iv) {
    uint64_t idx = nb + jl;
    idx = idx < args.n ? idx : args.n - 1;
    r = load_ext_raw(args, idx);
    iv = init ? reinterpret_cast<gptr_u32>(reinterpret_cast<uint64_t>(init))[idx] : 0u;
  };

  // wave cursor: unit ordinal `cur_o` of block `cur_b` is the next unassigned unit
  uint64_t cur_b = b_lo;
  uint32_t cur_o = 0;
  uint64_t range_hi = b_hi;  // end of the range being walked
  ExtRaw rj = {0, 0};
  uint32_t ivj = 0;
  if (b_lo < b_hi) prefetch(cur_b, rj, ivj);
  if (load_tables) load_lds_tables(g_lds, dc);  // overlaps the first extents' latency
  if constexpr (kExt == kExtLogHeaders) log_length(args, rj);

  // The block still open at the end of the last retired round and the xor of
  // its units so far (wave-uniform); ~0 = none.
  uint32_t carry_b = ~0u;  // block index relative to b_lo
  uint32_t carry_v = 0;
  // the previous round: braids, unit and block, and what its finish needs
  uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;
  u32x4 pshift = {0, 0, 0, 0}, pfin = {0, 0, 0, 0};
  uint32_t paux0 = 0, paux1 = 0;
  (void)paux1;  // (two-load A/B builds only)
  uint64_t pk = 0, pb = 0, pat = 0;
  bool pact = false, plast = false, pfits = true, pfast = false;

  uint64_t pend_a = 0;  // this lane's parked result (0 = none), see retire()
  uint32_t pend_v = 0, pend_i = 0;
  uint32_t round = 0;   // rounds retired so far (wave-uniform)
  // Bad records are counted wave-uniform (one ballot per round, in converged
  // code, so the count lives in an SGPR) and added to *nbad once per walk: one
  // atomic per bad block on one address serialises at the memory side (a
  // batch of 1M bad blocks took 8.7 ms instead of 0.65), and a per-lane count
  // was one VGPR too many -- the SSTable walks spilled (round 6).
  uint32_t nbad_w = 0;
  auto retire = [&]() {
    const uint32_t raw = merge_braids(g_lds, p0, p1, p2, p3, lane_fin);
    uint32_t v = raw;
    if (!pfast) {  // (a fast round: 8 whole blocks, no shift, no sum, no carry)
      v = cols_apply(pshift, raw, li);  // A^(128 (k mod 512))
      if (pk >= kShiftCols) v = shift_rows(g_lds, dc, v, pk & ~(uint64_t)(kShiftCols - 1));
      v = pact ? v : 0u;
      const uint32_t key = pact ? (uint32_t)(pb - b_lo) : ~0u;  // a wave's blocks span < 2^32
      // segmented inclusive xor-scan over the 8 groups (blocks non-decreasing in g)
#pragma unroll
      for (uint32_t d = 8; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, d);
        const uint32_t tk = (uint32_t)__shfl_up((int)key, d);
        if (lane >= d && tk == key) v ^= t;
      }
      if (pact && key == carry_b) v ^= carry_v;
      // the block open after group 7 carries into the next round
      const uint32_t key7 = __builtin_amdgcn_readlane(key, 56);
      const uint32_t last7 = __builtin_amdgcn_readlane((uint32_t)plast, 56);
      carry_v = __builtin_amdgcn_readlane(v, 56);
      carry_b = (key7 != ~0u && !last7) ? key7 : ~0u;
    }
    // finish: register after the block = A^-z(v) (A^(1-z) for the seal's type byte)
    const uint32_t l = cols_apply(pfin, v, li);
    const uint32_t crc = l ^ 0xffffffffu;
    // this round's bad records (a group's lanes agree; lane 0 of the group counts)
    bool good = true;
    if constexpr (mode == kModeSstSeal || mode == kModeSstCrc || mode == kModeLogSeal) {
      good = pfits;
    } else if constexpr (mode == kModeVerify) {
      good = ((args.flags & 1u) ? mask_crc(crc) : crc) == paux0;
    } else if constexpr (mode != kModeOut) {  // kModeSstVerify (table/format.cc:95-103), kModeLogVerify (log_reader.cc:228-242)
#ifndef LSBM_VERIFY_TWO_LOADS
      good = pfits && unmask_crc(paux0) == crc;
#else
      good = pfits && unmask_crc(unaligned_word(paux0, paux1, pat)) == crc;
#endif
    }
    if constexpr (mode != kModeOut)
      nbad_w += (uint32_t)__builtin_popcountll(__ballot(pact && plast && li == 0u && !good));
    // The finishing group's result is parked in ONE lane of the group, the
    // lane whose index is the round number mod 8, and written by
    // flush_stores() once every 8 rounds: stores count in the same in-order
    // vmcnt queue as loads, and a store in front of row loads delays every
    // wait for those rows until it is acknowledged (~3,000 cycles with every
    // CU streaming), so one flush per 8 rounds instead of a store per round.
    if (!(pact && plast)) return;
    const bool mine = li == (round & 7u);
    if constexpr (mode == kModeSstSeal) {  // table/table_builder.cc:245-249
      if (!pfits) return;
      const uint32_t typ = paux0 & 0xffu;
      const uint32_t m = mask_crc((l ^ advance_byte(typ)) ^ 0xffffffffu);  // Extend(crc, &type, 1)
      // the trailer [type][masked crc LE32] at pat, one byte per lane.  These
      // scattered writes cost ~13% of HBM peak (A/B: the same 4-byte writes
      // added to verify took it from 75% to 62%; whole 64-B line writes were
      // no better): lsbm_sst_trailer_crcs_dev returns dense CRCs instead.
      // (non-temporal stores, and no-return atomic and/or merges of whole
      // words: no different, A/B; lsbm_sst_seal_dev uses this mode only
      // when it cannot have scratch for its two-pass seal)
      if (li < kTrailer)
        reinterpret_cast<uint8_t*>(pat)[li] = (uint8_t)(li == 0 ? typ : m >> (8 * (li - 1)));
    } else if constexpr (mode == kModeSstCrc) {  // the same crc, dense: out[b]
      const uint32_t typ = paux0 & 0xffu;
      if (mine) {
        pend_a = reinterpret_cast<uint64_t>(args.out + pb);
        pend_v = pfits ? mask_crc((l ^ advance_byte(typ)) ^ 0xffffffffu) : 0u;
      }
    } else if constexpr (mode == kModeLogSeal) {  // log::Writer::EmitPhysicalRecord, common/log_writer.cc:85-88
      if (!pfits && li == 0 && args.out) args.out[pb] = 0;
      if (pfits && mine) {  // header[0..4) at pat (+ out[pb] when requested)
        pend_a = pat;
        pend_v = mask_crc(crc);
        pend_i = (uint32_t)(pb - b_lo);
      }
    } else if constexpr (mode == kModeOut) {
      if (mine) {
        pend_a = reinterpret_cast<uint64_t>(args.out + pb);
        pend_v = (args.flags & 1u) ? mask_crc(crc) : crc;
      }
    } else {  // verify modes: good (above)
#ifdef LSBM_DIAG_VERIFY_WRITEBACK  // diagnostic builds only: rewrite the stored crc bytes
      if (pfits && li < 4)
        reinterpret_cast<uint8_t*>(pat)[li] = (uint8_t)(paux0 >> (8 * li));
#endif
      if (mine) {
        pend_a = reinterpret_cast<uint64_t>(args.ok + pb);
        pend_v = good ? 1u : 0u;
      }
    }
  };
  auto flush_stores = [&]() {
#ifndef LSBM_DIAG_NO_STORE  // diagnostic builds only: results not written
    if (pend_a) {
      if constexpr (mode == kModeSstSeal) {
        uint8_t* t = reinterpret_cast<uint8_t*>(pend_a & 0x00ffffffffffffffull);
        t[0] = (uint8_t)(pend_a >> 56);
        t[1] = (uint8_t)pend_v;
        t[2] = (uint8_t)(pend_v >> 8);
        t[3] = (uint8_t)(pend_v >> 16);
        t[4] = (uint8_t)(pend_v >> 24);
      } else if constexpr (mode == kModeLogSeal) {
        if (args.file) {  // (null: the masked crcs only, lsbm_log_crcs_dev)
#ifndef LSBM_LOG_BYTE_STORES  // A/B builds only
          // header[0..4) as one unaligned dword store (gfx950 global memory
          // takes any byte alignment) instead of four byte stores: every store
          // sits in the vmcnt queue in front of the next rounds' row loads
          typedef __attribute__((address_space(1), aligned(1))) uint32_t* gu32u;
          *reinterpret_cast<gu32u>(pend_a) = pend_v;
#else
          uint8_t* h = reinterpret_cast<uint8_t*>(pend_a);
          h[0] = (uint8_t)pend_v;
          h[1] = (uint8_t)(pend_v >> 8);
          h[2] = (uint8_t)(pend_v >> 16);
          h[3] = (uint8_t)(pend_v >> 24);
#endif
        }
        if (args.out) args.out[b_lo + pend_i] = pend_v;
      } else if constexpr (mode == kModeOut || mode == kModeSstCrc) {
        *reinterpret_cast<uint32_t*>(pend_a) = pend_v;
      } else {
        *reinterpret_cast<uint8_t*>(pend_a) = (uint8_t)pend_v;
      }
    }
#endif
    pend_a = 0;
  };

  while (cur_b < range_hi) {
    // The round's prologue at raised wave priority (round 6): from the end of
    // the last round's rows to this round's first row loads the wave has no
    // row loads in flight, while the other waves of its SIMD stream at normal
    // priority; at s_setprio 2 it takes the issue slots until it has absorbed
    // this round's first kPrioRows rows.  A/B, same box: SSTable verify /
    // trailer CRCs / seal +2-2.5 points of HBM peak at 16 rows (8: +1.5-1.9;
    // 24: 0.2-0.4 less; 32, near a whole round: 1.5 less; only until the
    // first loads: +0.2-0.4); the fixed kernel, whose group
    // prologue is short, and the stream kernel's sub-piece set-up or tail
    // (config 4 -0.7 to -2) gain nothing (profiles/r06/events_ab/prio_*.log).
    __builtin_amdgcn_s_setprio(2);
    // Find the 8 groups' units in one round: lane j holds block cur_b + j
    // (8 units never span more than 9 blocks), an inclusive prefix sum over
    // the lanes' unit counts, then one ballot per group.  ALU + shuffles only:
    // the extents arrived during the previous round.
    uint64_t sj = 0, ej = 0, atj = 0;
    bool fj = true;
    extent_from_raw(args, cur_b + lane, rj, sj, ej, fj, atj);
    const Frame ft = frame_of(sj, ej, kMaxRows);
    const bool vj = lane < 9u && cur_b + lane < range_hi;
    const uint32_t units_j = vj ? ft.units : 0u;
    // Fast round: the cursor is at a block start and the next 8 blocks are
    // one unit each, so group g takes block cur_b + g (every round over an
    // SSTable's data blocks).  Wave-uniform.
    const bool fast = cur_o == 0u && __ballot(lane < 8u && units_j == 1u) == 0xffull;
    uint32_t jg = g, jnext = 8, pre_before = g, pre8 = 8;
    if (!fast) {
      uint32_t pre = units_j;
#pragma unroll
      for (uint32_t d = 1; d < 16; d <<= 1) {  // lanes >= 9 contribute 0: a 16-lane scan suffices
        const uint32_t t = (uint32_t)__shfl_up((int)pre, d, 16);
        if ((lane & 15u) >= d) pre += t;
      }
      jg = 0;
      jnext = 0;
#pragma unroll
      for (uint32_t q = 0; q < 9; q++) {
        // count of lanes (among the first 9) whose prefix <= cur_o + q
        const uint64_t m = __ballot((lane < 9) && pre <= cur_o + q);
        const uint32_t c = (uint32_t)__builtin_popcountll(m);
        if (q == g) jg = c;
        if (q == 8) jnext = c;
      }
      // shuffles run with every lane active (a bpermute from an inactive
      // source lane reads 0), then select
      const uint32_t pre_prev = (uint32_t)__shfl((int)pre, (int)(jg ? jg - 1 : 0));
      pre_before = jg ? pre_prev : 0u;
      const uint32_t pre8_prev = (uint32_t)__shfl((int)pre, (int)(jnext ? jnext - 1 : 0));
      pre8 = jnext ? pre8_prev : 0u;
    }
    const uint32_t my_t = cur_o + g;  // this group's unit, as an offset from the cursor
    const uint64_t b = cur_b + jg;
    const bool active = jg < 9 && b < range_hi;
    Frame f = {0, 0, 0, 1, 1, 1, 0};
    f.s = __shfl((unsigned long long)ft.s, (int)jg);
    f.e = __shfl((unsigned long long)ft.e, (int)jg);
    f.row0 = __shfl((unsigned long long)ft.row0, (int)jg);
    f.rows = __shfl((unsigned long long)ft.rows, (int)jg);
    f.units = (uint32_t)__shfl((int)ft.units, (int)jg);
    f.q = (uint32_t)__shfl((int)ft.q, (int)jg);
    f.rem = (uint32_t)__shfl((int)ft.rem, (int)jg);
    const uint32_t iv = (uint32_t)__shfl((int)ivj, (int)jg);
    const bool fits = __shfl((int)fj, (int)jg) != 0;
    const uint64_t at = __shfl((unsigned long long)atj, (int)jg);
    const uint32_t o = my_t - pre_before;
    // the cursor after these 8 units, and the next round's extents
    uint64_t nb = cur_b + jnext;
    uint32_t no = cur_o + 8 - pre8;
    uint64_t next_hi = range_hi;
    if (chunked && nb >= range_hi) {  // (wave-uniform) this range is done: the next piece's
      if (!advance(nb, next_hi)) nb = next_hi = range_hi;  // (none left: done)
      no = 0;
    }
    ExtRaw rn;
    uint32_t ivn;
    prefetch(nb, rn, ivn);

    uint32_t rows = 0;
    uint64_t k = 0;  // rows of the frame after this unit
    uint64_t row_a = dummy;  // absolute address of this lane's slice of the unit's first row
    uint64_t r0 = 0;
    // rows whose loads are inside [s, e): [r_lo, r_hi).  Per lane at most two
    // rows need a fix (fix_word): rfs, whose chunk starts before s and holds
    // init bytes of [s-4, s) or straddles s (s - chunk in [1, 19]), and rfe,
    // whose chunk straddles e (e - chunk in [1, 15]).  ds / de: s / e relative
    // to the chunk (-64 / 64: no cut).
    uint32_t r_lo = 0, r_hi = 0, rfs = ~0u, rfe = ~0u;
    int32_t ds = -64, de_s = 64, de_e = 64;
    if (active) {
      // balanced units: a 4,118-B SSTable block (33-34 rows) is 17 + 17 rows,
      // not 2 + 32, so a round of 8 such units runs 17 row steps, not 32
      const uint64_t start = (uint64_t)o * f.q + (o < f.rem ? o : f.rem);
      rows = f.q + (o < f.rem ? 1u : 0u);
      r0 = f.row0 + start;
      row_a = r0 * kRowBytes + 16u * li;
      k = f.rows - start - rows;
      const bool edge = r0 * kRowBytes < f.s || (r0 + rows) * kRowBytes > f.e;
      r_hi = rows;
      if (edge) {
        r_lo = r_hi = 0;
        if (f.s < f.e) {
          const int64_t dl = (int64_t)f.s - 16 - (int64_t)row_a;  // chunk end > s
          const int64_t dh = (int64_t)f.e - (int64_t)row_a;       // chunk start < e
          const int64_t lo = dl < 0 ? 0 : dl / (int64_t)kRowBytes + 1;
          const int64_t hi = dh <= 0 ? 0 : (dh + kRowBytes - 1) / (int64_t)kRowBytes;
          r_lo = (uint32_t)(lo < (int64_t)rows ? lo : rows);
          r_hi = (uint32_t)(hi < (int64_t)rows ? hi : rows);
        }
        const int64_t t_s = (int64_t)f.s - 1 - (int64_t)row_a;
        if (t_s >= 0 && (t_s & 127) < 19 && (t_s >> 7) < (int64_t)rows) {
          rfs = (uint32_t)(t_s >> 7);
          ds = (int32_t)(t_s & 127) + 1;
          const int64_t ee = (int64_t)f.e - (int64_t)(row_a + (uint64_t)rfs * kRowBytes);
          de_s = ee < 64 ? (int32_t)ee : 64;
        }
        // (only for a non-empty block: the chunk of byte e - 1 must overlap [s, e),
        // or an empty block at the start of an allocation would read before it)
        const int64_t t_e = (int64_t)f.e - 1 - (int64_t)row_a;
        if (f.s < f.e && t_e >= 0 && (t_e & 127) < 15 && (t_e >> 7) < (int64_t)rows &&
            (uint32_t)(t_e >> 7) != rfs) {
          rfe = (uint32_t)(t_e >> 7);
          de_e = (int32_t)(t_e & 127) + 1;
          // that chunk is read ONCE, by the early load below, never by the row
          // loop: its bytes >= e may be another block's trailer or log header,
          // which a seal in another wave can be writing right now, so two
          // reads of it need not agree
          r_hi = rfe;
        }
      }
    }
    // What this round's finish needs is loaded after its rows and used one
    // round later, behind the next round's first row loads (every load
    // unconditional, from a valid address): the columns of A^(128 (k mod 512))
    // and of A^-z / A^(1-z); expect[b] (verify), types[b] (seal), or the two
    // aligned dwords holding a stored trailer / log header crc (verifies).
    // Until then only these compact words stay live across the row loop.
    const bool last = active && o + 1 == f.units;
    const uint32_t zf = (uint32_t)((f.row0 + f.rows) * kRowBytes - f.e);  // < 128
    const uint32_t fin_i = active ? (mode == kModeSstSeal || mode == kModeSstCrc ? 128u : 127u) - zf : 127u;
    const uint32_t st_i = (active ? (uint32_t)(k & (kShiftCols - 1)) : 0u) | (fin_i << 16) |
                          (last ? 1u << 24 : 0u) | (fits ? 1u << 25 : 0u) | (active ? 1u << 26 : 0u);
    const uint32_t b_rel = (uint32_t)(b - b_lo);  // a wave's blocks span < 2^32
    const uint32_t k_hi = (uint32_t)(k >> 9);     // shift beyond the columns (blocks > 64 KiB)

    // uniform trip count: the longest unit of the 8 groups
    uint32_t rows_max = rows;
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 8));
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 16));
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 32));
    rows_max = __builtin_amdgcn_readfirstlane(rows_max);
    // ... and, in the SSTable modes, the shortest (0 with an idle group):
    // rows 1 .. rows_min - 2 of every unit are whole rows of its block, loaded
    // without the select below.  (A/B, profiles/r02/ab/s66_row_fast.log: SST
    // verify / trailer CRCs +1.3-1.5 points, where a round is 8 blocks of 33-34
    // rows; config 4 -1.5 and WAL records -1.3, where rows_min is mostly small
    // and the test costs more than it saves.)
#ifndef LSBM_NO_ROW_FAST  // A/B builds only
    constexpr bool kRowFast = kMode == kModeSstSeal || kMode == kModeSstVerify || kMode == kModeSstCrc;
#else
    constexpr bool kRowFast = false;
#endif
    uint32_t rows_min = 0;
    if constexpr (kRowFast) {
      rows_min = active ? rows : 0u;
      rows_min = min(rows_min, (uint32_t)__shfl_xor((int)rows_min, 8));
      rows_min = min(rows_min, (uint32_t)__shfl_xor((int)rows_min, 16));
      rows_min = min(rows_min, (uint32_t)__shfl_xor((int)rows_min, 32));
      rows_min = __builtin_amdgcn_readfirstlane(rows_min);
    }

    // Row r of this lane is loaded from its address when r in [r_lo, r_hi),
    // else from the zero pad.  Branch-free select, and the address pinned in
    // every lane: where a lane's value is dead, hipcc otherwise left that
    // lane's address undefined although the wave still issues the load
    // (observed: reads below the batch, a GPU fault).
    //
    // Rows 1 .. rows_min - 2 (SSTable modes; a wave-uniform test) need no
    // select: only a unit's row 0 can hold chunks before s (r_lo <= 1) and only
    // its last row chunks at or past e (r_hi >= rows - 1), so there every
    // lane's chunk is in [s, e) and the address is the row's own.
    auto row_addr = [&](uint32_t r) -> gptr_u32x4 {
      if constexpr (kRowFast) {
        if (r >= 1u && r + 1u < rows_min) {
          uint64_t p = row_a + (uint64_t)r * kRowBytes;
          asm volatile("" : "+v"(p));
          return reinterpret_cast<gptr_u32x4>(p);
        }
      }
      const bool ok = (r >= r_lo) & (r < r_hi);
      uint64_t p = ok ? row_a + (uint64_t)r * kRowBytes : dummy;
      asm volatile("" : "+v"(p));
      return reinterpret_cast<gptr_u32x4>(p);
    };
    // two banks of 4 rows, loads always issued (pad reads past the unit) so
    // that the loads in flight are counted exactly
    u32x4 ba[4], bb[4];
#pragma unroll
    for (uint32_t k2 = 0; k2 < 4; k2++) ba[k2] = __builtin_nontemporal_load(row_addr(k2));
    // the chunk straddling e sits in the unit's last row (rfe = rows - 1): the
    // row loop absorbs zeros for it, and its bytes < e are added after the
    // loop (below) from this one copy
    uint64_t pe = rfe != ~0u ? row_a + (uint64_t)rfe * kRowBytes : dummy;
    asm volatile("" : "+v"(pe));
    const u32x4 wl = *reinterpret_cast<gptr_u32x4>(pe);

    // while those loads fly: the init bytes and the previous round's retire
    const uint32_t u = (kExt != kExtLogHeaders && init) ? nib_lds_at(g_lds, kNibNeg4, iv ^ 0xffffffffu)  // A^-4(init ^ ~0)
                            : args.u_noinit;
    retire();
#ifdef LSBM_FLUSH_EVERY_ROUND  // A/B builds only
    flush_stores();
#else
    if ((round & 7u) == 7u) flush_stores();
#endif
    round++;

    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    auto absorb = [&](u32x4 w, uint32_t r) {  // rows read from the pad are zero
      // Consume the loaded row in straight-line code: with the only use inside
      // the (r < rows) branch, the vmcnt wait sat on that path alone, and the
      // next reload of the bank had to drain every load still in flight.
      asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w));
      if (r < rows) STEP_ROW(w);
    };
    // The start fix (init bytes, bytes before s) only ever falls on rows 0
    // and 1 of a unit: chunk c of row 0 has c <= s - 4 and the fix chunk has
    // c >= s - 19.
    auto absorb_start = [&](u32x4 w, uint32_t r) {
      if (rfs == r) {
        w.x = fix_word(w.x, ds, de_s, u, 0);
        w.y = fix_word(w.y, ds, de_s, u, 4);
        w.z = fix_word(w.z, ds, de_s, u, 8);
        w.w = fix_word(w.w, ds, de_s, u, 12);
      }
      absorb(w, r);
    };
    // Every bank load is unconditional (rows past the unit read the pad): with
    // a load skipped on one path, the vmcnt waits after the merge point must
    // assume the shorter queue and over-wait on the other path.
#pragma unroll
    for (uint32_t k2 = 0; k2 < 4; k2++) bb[k2] = __builtin_nontemporal_load(row_addr(4 + k2));
    absorb_start(ba[0], 0);
    absorb_start(ba[1], 1);
    absorb(ba[2], 2);
    absorb(ba[3], 3);
    // Log headers: the next round's record lengths.  Their header offsets were
    // loaded before this round's first row bank, so they have landed by now
    // (vmcnt retires in order); issued right behind the offsets, the dependent
    // load made every round wait out a memory latency with no row loads in
    // flight (A/B: +1.2 points on every log mode, profiles/r02/ab/s55_*).
    if constexpr (kExt == kExtLogHeaders) log_length(args, rn);
    // End fix.  The register kept per braid is the pre-lookup word c = s ^ w
    // of the last row absorbed, and the row loop absorbed w = 0 for the chunk
    // straddling e, so adding its bytes < e is a plain xor after the loop:
    // c ^= w & keep (lanes without rfe loaded the zero pad: 0).  Computed
    // here, pinned, so that no wait follows the loop.
    uint32_t dx = wl.x & low_bytes(min(max(de_e, 0), 4));
    uint32_t dy = wl.y & low_bytes(min(max(de_e - 4, 0), 4));
    uint32_t dz = wl.z & low_bytes(min(max(de_e - 8, 0), 4));
    uint32_t dw = wl.w & low_bytes(min(max(de_e - 12, 0), 4));
    asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz), "+v"(dw));
    // fully unrolled (rows_max <= kMaxRows): a rolled loop got a vmcnt(0) at
    // its header, draining the bank in flight every 8 rows
#pragma unroll
    for (uint32_t r = 4; r < kMaxRows; r += 8) {
      if (r >= rows_max) break;
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) ba[k2] = __builtin_nontemporal_load(row_addr(r + 4 + k2));
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) absorb(bb[k2], r + k2);
      if (r + 4 == kPrioRows) __builtin_amdgcn_s_setprio(0);
      if (r + 4 >= rows_max) break;
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) bb[k2] = __builtin_nontemporal_load(row_addr(r + 8 + k2));
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) absorb(ba[k2], r + 4 + k2);
      if (r + 8 == kPrioRows) __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_s_setprio(0);  // (a round of fewer rows)
    c0 ^= dx;
    c1 ^= dy;
    c2 ^= dz;
    c3 ^= dw;
    // this round becomes the previous one
    p0 = c0;
    p1 = c1;
    p2 = c2;
    p3 = c3;
    pfast = fast;
    pact = (st_i >> 26) & 1u;
    plast = (st_i >> 24) & 1u;
    pfits = (st_i >> 25) & 1u;
    pb = b_lo + b_rel;
    pk = ((uint64_t)k_hi << 9) | (st_i & 0x1ffu);
    pat = at;
    {
      const uint32_t ks = st_i & 0xffffu, fi = (st_i >> 16) & 0xffu;
      pshift = *reinterpret_cast<gptr_u32x4>(reinterpret_cast<uint64_t>(&dc->shift_cols[ks][4 * li]));
      pfin = *reinterpret_cast<gptr_u32x4>(reinterpret_cast<uint64_t>(&dc->fin_cols[fi][4 * li]));
      const bool need = plast && pfits;
      uint64_t q0 = dummy, q1 = dummy;
      if constexpr (mode == kModeVerify) {
        q0 = need ? reinterpret_cast<uint64_t>(args.expect + pb) : dummy;
      } else if constexpr (mode == kModeSstSeal || mode == kModeSstCrc) {
        q0 = need ? reinterpret_cast<uint64_t>(args.types + pb) : dummy;
      } else if constexpr (mode == kModeSstVerify || mode == kModeLogVerify) {
#ifndef LSBM_VERIFY_TWO_LOADS  // A/B builds only
        // the stored crc [pat, pat + 4) as one unaligned dword load
        q0 = need ? pat : dummy;
#else
        // the dwords holding bytes pat and pat + 3 (one dword when aligned:
        // never a byte past the stored crc)
        q0 = need ? (pat & ~3ull) : dummy;
        q1 = need ? ((pat + 3) & ~3ull) : dummy;
#endif
      }
      asm volatile("" : "+v"(q0), "+v"(q1));
      if constexpr (mode == kModeSstSeal || mode == kModeSstCrc) {
        paux0 = *reinterpret_cast<gptr_u8>(q0);
      } else if constexpr (mode == kModeVerify) {
        paux0 = *reinterpret_cast<gptr_u32>(q0);
      } else if constexpr (mode == kModeSstVerify || mode == kModeLogVerify) {
#ifndef LSBM_VERIFY_TWO_LOADS
        typedef const __attribute__((address_space(1), aligned(1))) uint32_t* gptr_u32u;
        paux0 = *reinterpret_cast<gptr_u32u>(q0);
#else
        paux0 = *reinterpret_cast<gptr_u32>(q0);
        paux1 = *reinterpret_cast<gptr_u32>(q1);
#endif
      }
    }
    rj = rn;
    ivj = ivn;
    cur_b = nb;
    cur_o = no;
    range_hi = next_hi;
  }
  retire();
  flush_stores();
  if (args.nbad && lane == 0 && nbad_w) atomicAdd(args.nbad, nbad_w);
}

}  // namespace lsbm
