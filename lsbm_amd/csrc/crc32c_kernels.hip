// crc32c_kernels.hip -- gfx950 kernels of the batched CRC-32C engine.
//
// crc32c_fixed_kernel   fixed-stride, len % 128 == 0, 16-B aligned blocks
//                       (SSTable-sized 4 KiB and 64 KiB batches; the headline)
// crc32c_units_kernel   any extents, any alignment (offsets[] batches, verify,
// crc32c_finish_kernel  SSTable trailer seal / verify): 32-row units per lane
//                       group, partial CRCs xor-ed per block, then finished
// fill_splitmix64_kernel, stream_read_kernel   benchmark helpers
//
// Both CRC kernels compute, per block, exactly what lsbm's
// crc32c::Extend(init, block, n) returns (util/crc32c.cc:286-329): the
// register starts at init ^ ~0 (:289), absorbs the bytes, and is inverted
// again (:328).  They differ from the reference only in how the bytes are
// absorbed (braids of A^128 steps instead of one serial A^4 chain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"

namespace lsbm {

__shared__ uint32_t g_lds[kLdsWords];

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Global-address-space pointer: addresses built from integers would otherwise
// be generic (flat) loads, which count on lgkmcnt too and force full drains.
typedef const __attribute__((address_space(1))) u32x4* gptr_u32x4;

#ifdef LSBM_DIAG_STAMPS  // diagnostic builds only (tools/ablate.sh): per-wave timeline
__device__ uint64_t g_stamps[4][65536];  // start, first-data, end, xcc id
extern "C" __attribute__((visibility("default"))) int lsbm_diag_stamps(uint64_t* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(uint64_t) * 4 * 65536) == hipSuccess ? 0 : -1;
}
#define DIAG_STAMP(k) do { if (lane == 0) g_stamps[k][wave & 65535] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define DIAG_STAMP(k) do { } while (0)
#endif

#ifndef LSBM_PF
#define LSBM_PF 4
#endif
constexpr uint32_t kPF = LSBM_PF;  // rows per load bank

constexpr int kAuxNT = 2;     // buffer-load cache policy: non-temporal (read-once stream)

// Issue the loads of rows [r0, r0 + kPF) of this lane's slice into bank X.
// Rows past the end re-read the last row (clamped, a cache hit), so the
// number of loads in flight is static and the compiler's vmcnt waits exact.
#define LOAD_BANK(X, r0)                                                          \
  do {                                                                            \
    _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPF; k_++) {                     \
      const uint32_t rr_ = (r0) + k_ < rows ? (r0) + k_ : rows - 1;               \
      X[k_] = __builtin_bit_cast(                                                 \
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, loff + rr_ * kRowBytes, 0, \
                                                       kAuxNT));                  \
    }                                                                             \
  } while (0)

// c_m = A^128(c_m) ^ w_m for the four braids of one 16-B row slice.
#define STEP_ROW(W)                                           \
  do {                                                        \
    c0 = row_step(g_lds, c0, (W).x, L0, L1, L2, L3);          \
    c1 = row_step(g_lds, c1, (W).y, L0, L1, L2, L3);          \
    c2 = row_step(g_lds, c2, (W).z, L0, L1, L2, L3);          \
    c3 = row_step(g_lds, c3, (W).w, L0, L1, L2, L3);          \
  } while (0)

// Absorb the rows of bank X that exist (rows r0 .. r0+kPF-1).
#define ABSORB(X, r0)                                                       \
  do {                                                                      \
    _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPF; k_++) {               \
      if ((r0) + k_ < rows) STEP_ROW(X[k_]);                                \
    }                                                                       \
  } while (0)

// ---------------------------------------------------------------------------
// Fixed-stride kernel.  Each wave takes 8 consecutive blocks at a time (one per
// 8-lane group); waves stride through the batch.  rows = len / 128.
// ---------------------------------------------------------------------------
template <bool kHasInit, uint32_t kRows>
__global__ __launch_bounds__(kBlockThreads) void crc32c_fixed_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t rows_arg, uint64_t n_blocks,
    const uint32_t* __restrict__ init, uint32_t* __restrict__ out, uint32_t flags,
    uint32_t k_value /* A^len(~0) ^ ~0: the init term of crc32c::Value */,
    const DevConsts* __restrict__ dc) {
  const uint32_t rows = kRows ? kRows : rows_arg;  // kRows != 0: fully unrolled
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = (lane & 31u) << 2;
  const uint32_t L0 = lb, L1 = lb | 0x80u, L2 = lb | 0x10000u, L3 = lb | 0x10080u;
  const uint32_t lane_fin = kNibFin | lb;
  const uint32_t wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg + wave_in_wg;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  const uint64_t ngroups = (n_blocks + 7) / 8;

  // The first group's first two banks are requested from HBM before the LDS
  // tables are filled, so the table fill hides under the first HBM latency.
  u32x4 a[kPF], b[kPF];
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t loff;
  auto set_group = [&](uint64_t grp) {
    const uint64_t blk = grp * 8 + g;
    // wave-uniform descriptor over the group's 8 blocks; per-lane 32-bit
    // offset (host guarantees 8 * stride < 2^32).  Lanes past the end re-read
    // block 0 of the group and discard the result.
    // num_records = the bytes of this group's blocks that exist: a load past
    // them returns zeros instead of touching memory beyond the batch
    const uint64_t nb = n_blocks - grp * 8 < 8 ? n_blocks - grp * 8 : 8;
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + grp * 8 * stride),
                                             (short)0, (int)((nb - 1) * stride + rows * kRowBytes),
                                             0x00020000);
    loff = (blk < n_blocks ? g : 0u) * (uint32_t)stride + 16u * li;
    asm volatile("" : "+v"(loff));  // defined in every lane (see crc32c_units_kernel)
  };
  // Static interleave: wave w takes groups w, w + nwaves, ...  At any moment
  // the GPU streams one contiguous ~128 MiB window of the batch.  (A dynamic
  // per-XCC work queue evened out per-wave finish times but was 5% slower
  // end to end: DESIGN.md section 4.)
  uint64_t grp = wave;
  DIAG_STAMP(0);
  if (grp < ngroups) {
    set_group(grp);
    LOAD_BANK(a, 0);
    if (kRows == 0 || kPF < rows) LOAD_BANK(b, kPF);
  }
  load_lds_tables(g_lds, dc);
  DIAG_STAMP(1);

  bool first = true;
  for (; grp < ngroups; grp += nwaves) {
    const uint64_t blk = grp * 8 + g;
    const bool valid = blk < n_blocks;
    // Two banks of kPF rows: while one bank is absorbed the other's loads
    // are in flight.  Row 0 initialises the braids (c = w); every later row
    // is c = A^128(c) ^ w.
    if (!first) {
      set_group(grp);
      LOAD_BANK(a, 0);
      if (kRows == 0 || kPF < rows) LOAD_BANK(b, kPF);
    }
    first = false;
    uint32_t c0 = a[0].x, c1 = a[0].y, c2 = a[0].z, c3 = a[0].w;
#pragma unroll
    for (uint32_t k = 1; k < kPF; k++)
      if (k < rows) STEP_ROW(a[k]);
    uint32_t r = kPF;
    while (r < rows) {
      if (kRows == 0 || r + kPF < rows) LOAD_BANK(a, r + kPF);
      ABSORB(b, r);
      r += kPF;
      if (r >= rows) break;
      if (kRows == 0 || r + kPF < rows) LOAD_BANK(b, r + kPF);
      ABSORB(a, r);
      r += kPF;
    }
#ifdef LSBM_ABL_NO_MERGE  // diagnostic builds only (tools/ablate.sh)
    const uint32_t raw = c0 ^ c1 ^ c2 ^ c3;
#else
    const uint32_t raw = merge_braids(g_lds, c0, c1, c2, c3, lane_fin);
#endif
    if (li == 7u && valid) {
      uint32_t crc;
      if (kHasInit)
        crc = raw ^ advance_glb(dc, init[blk] ^ 0xffffffffu, (uint64_t)rows * kRowBytes) ^
              0xffffffffu;
      else
        crc = raw ^ k_value;
      out[blk] = (flags & 1u) ? mask_crc(crc) : crc;
    }
  }
  DIAG_STAMP(2);
#ifdef LSBM_DIAG_STAMPS
  if (lane == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    g_stamps[3][wave & 65535] = xcc;
  }
#endif
}
// ---------------------------------------------------------------------------
// Ragged path: units kernel + finish kernel.
//
// Frame.  Rows are 128-B aligned in the absolute address space, so every load
// is an aligned 16-B load whatever the block's alignment.  For block [s, e):
//   * bytes of the frame outside [s, e) are zero; leading zeros leave a raw
//     CRC unchanged, so the frame may start early for free;
//   * the init register v = init ^ ~0 is injected as 4 virtual bytes
//     u = A^-4(v) at [s-4, s) (absorbing u from zero gives exactly v);
//   * the frame ends z = frame_end - e bytes late: undone with A^-z.
// Units.  The frame is cut into units of <= 32 rows (crc32c_types.h).  Each
// wave walks a contiguous range of blocks and hands the next 8 units of the
// range to its 8 lane groups, so most steps are uniform 32-row loops whatever
// the block lengths.  A unit's raw CRC, shifted to the frame end by
// A^(4096 k), is xor-ed into acc[block]; the finish kernel turns acc into
// the CRC and applies the output mode.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t frame_word(uint32_t raw, uint64_t a, uint64_t s, uint64_t e,
                                               uint32_t u) {
  // keep the bytes of the dword at address a that lie in [s, e)
  const int64_t lo = (int64_t)s - (int64_t)a, hi = (int64_t)e - (int64_t)a;
  const uint32_t l = lo < 0 ? 0u : (lo > 4 ? 4u : (uint32_t)lo);
  const uint32_t h = hi < 0 ? 0u : (hi > 4 ? 4u : (uint32_t)hi);
  const uint64_t keep = h > l ? (((1ull << (8 * h)) - 1ull) & ~((1ull << (8 * l)) - 1ull)) : 0ull;
  uint32_t w = raw & (uint32_t)keep;
  // virtual init bytes u at [s-4, s)
  const int64_t d = (int64_t)a - ((int64_t)s - 4);
  if (d >= 0 && d < 4) w ^= u >> (8 * d);
  else if (d < 0 && d > -4) w ^= u << (8 * (-d));
  return w;
}

// Block b's extent [s, e) as absolute addresses.
__device__ __forceinline__ void block_extent(const RaggedArgs& a, uint64_t b, uint64_t& s,
                                             uint64_t& e) {
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  if (a.extents == kExtHandles) {
    const uint64_t off = a.handles[2 * b], sz = a.handles[2 * b + 1];
    s = base + off;
    e = s + sz + (a.mode == kModeSstVerify ? 1u : 0u);  // verify covers the type byte
  } else if (a.extents == kExtFixed) {
    s = base + b * a.stride;
    e = s + a.len;
  } else {
    s = base + a.offsets[b];
    e = base + a.offsets[b + 1];
    if (e < s) e = s;
  }
}

struct Frame {
  uint64_t s, e, row0, rows;  // rows >= 1
  uint32_t units;             // ceil(rows / 32)
};

__device__ __forceinline__ Frame block_frame(const RaggedArgs& a, uint64_t b) {
  Frame f;
  block_extent(a, b, f.s, f.e);
  f.row0 = (f.s - 4) >> 7;
  const uint64_t row_end = (f.e + 127) >> 7;
  f.rows = row_end > f.row0 ? row_end - f.row0 : 1;
  f.units = (uint32_t)((f.rows + kUnitRows - 1) / kUnitRows);
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

// A^(4096 k)(v): LDS tables for bits 0..15 of k, global ones beyond.
__device__ __forceinline__ uint32_t shift_units(const uint32_t* lds, const DevConsts* dc,
                                                uint32_t v, uint64_t k) {
  for (uint32_t i = 0; k; i++, k >>= 1)
    if (k & 1u) v = i < 16 ? nib_lds_at(lds, kNibU4096 + i * 512, v) : nib_glb(dc->pow_nib[12 + i], v);
  return v;
}

__global__ __launch_bounds__(kBlockThreads) void crc32c_units_kernel(RaggedArgs args) {
  const DevConsts* __restrict__ dc = args.dc;
  load_lds_tables(g_lds, dc);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = (lane & 31u) << 2;
  const uint32_t L0 = lb, L1 = lb | 0x80u, L2 = lb | 0x10000u, L3 = lb | 0x10080u;
  const uint32_t lane_fin = kNibFin | lb;
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  // this wave's contiguous range of blocks
  const uint64_t b_lo = args.n * wave / nwaves, b_hi = args.n * (wave + 1) / nwaves;
  const uint64_t dummy = reinterpret_cast<uint64_t>(dc->zero16);
#ifdef LSBM_DEBUG_BOUNDS
  if (threadIdx.x == 0 && blockIdx.x == 0)
    printf("units: n %lu base %lx dbg [%lx, %lx) acc %p dc %p dummy %lx grid %u\n", (unsigned long)args.n,
           (unsigned long)args.base, (unsigned long)args.dbg_lo, (unsigned long)args.dbg_hi, args.acc, dc,
           (unsigned long)dummy, gridDim.x);
#endif

  // wave cursor: unit ordinal `cur_o` of block `cur_b` is the next unassigned unit
  uint64_t cur_b = b_lo;
  uint32_t cur_o = 0;
  while (cur_b < b_hi) {
    // Find the 8 groups' units in one round: lane j reads block cur_b + j
    // (8 units never span more than 9 blocks), an inclusive prefix sum over
    // the lanes' unit counts, then one ballot per group.
    const uint64_t bj = cur_b + lane;
    Frame fj = {0, 0, 0, 1, 0};
    if (lane < 9 && bj < b_hi) fj = block_frame(args, bj);
    uint32_t pre = fj.units;
#pragma unroll
    for (uint32_t d = 1; d < 16; d <<= 1) {  // lanes >= 9 contribute 0: a 16-lane scan suffices
      const uint32_t t = (uint32_t)__shfl_up((int)pre, d, 16);
      if ((lane & 15u) >= d) pre += t;
    }
    const uint32_t my_t = cur_o + g;  // this group's unit, as an offset from the cursor
    uint32_t jg = 0, jnext = 0;
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
    const uint32_t pre_before = jg ? pre_prev : 0u;
    const uint64_t b = cur_b + jg;
    const bool active = jg < 9 && b < b_hi;
    Frame f = {0, 0, 0, 1, 1};
    f.s = __shfl((unsigned long long)fj.s, (int)jg);
    f.e = __shfl((unsigned long long)fj.e, (int)jg);
    f.row0 = __shfl((unsigned long long)fj.row0, (int)jg);
    f.rows = __shfl((unsigned long long)fj.rows, (int)jg);
    f.units = (uint32_t)__shfl((int)fj.units, (int)jg);
    const uint32_t o = my_t - pre_before;

    uint32_t rows = 0, k = 0;
    uint64_t row_a = dummy;  // absolute address of this lane's slice of the unit's first row
    // rows whose loads are inside [s, e): [r_lo, r_hi); rows needing the
    // masking / init-byte fix: rs0, rs1 (around s) and re (holding e - 1)
    uint32_t r_lo = 0, r_hi = 0, rs0 = ~0u, rs1 = ~0u, re = ~0u;
    uint32_t u = 0;
    if (active) {
      const uint32_t first_rows = (uint32_t)(f.rows - (uint64_t)kUnitRows * (f.units - 1));
      rows = o == 0 ? first_rows : kUnitRows;
      const uint64_t r0 = f.row0 + (o == 0 ? 0 : first_rows + (uint64_t)kUnitRows * (o - 1));
      row_a = r0 * kRowBytes + 16u * li;
      k = f.units - 1 - o;
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
        const int64_t rr0 = (int64_t)((f.s - 4) >> 7) - (int64_t)r0;
        const int64_t rr1 = (int64_t)((f.s - 1) >> 7) - (int64_t)r0;
        const int64_t rre = f.e > f.s ? (int64_t)((f.e - 1) >> 7) - (int64_t)r0 : -1;
        rs0 = rr0 >= 0 && rr0 < rows ? (uint32_t)rr0 : ~0u;
        rs1 = rr1 >= 0 && rr1 < rows ? (uint32_t)rr1 : ~0u;
        re = rre >= 0 && rre < rows ? (uint32_t)rre : ~0u;
      }
      if (r0 * kRowBytes < f.s) {  // the init bytes [s-4, s) may straddle two units
        const uint32_t v = (args.init ? args.init[b] : 0u) ^ 0xffffffffu;
        u = nib_glb(dc->neg4_nib, v);
      }
    }
    // uniform trip count: the longest unit of the 8 groups
    uint32_t rows_max = rows;
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 8));
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 16));
    rows_max = max(rows_max, (uint32_t)__shfl_xor((int)rows_max, 32));
    rows_max = __builtin_amdgcn_readfirstlane(rows_max);

    // Row r of this lane is loaded from its address when r in [r_lo, r_hi),
    // else from the zero pad.  Branch-free select, and the address pinned in
    // every lane: where a lane's value is dead, hipcc otherwise left that
    // lane's address undefined although the wave still issues the load
    // (observed: reads below the batch, a GPU fault).
    auto row_addr = [&](uint32_t r) -> gptr_u32x4 {
      const bool ok = (r >= r_lo) & (r < r_hi);
      uint64_t p = ok ? row_a + (uint64_t)r * kRowBytes : dummy;
#ifdef LSBM_DEBUG_BOUNDS  // diagnostic builds only: report and neutralise wild loads
      if (p != dummy && (p + 16 <= args.dbg_lo || p >= args.dbg_hi)) {
        printf("OOB wave %lu lane %u b %lu o %u r %u rows %u s %lx e %lx row_a %lx p %lx\n",
               (unsigned long)wave, lane, (unsigned long)b, o, r, rows, (unsigned long)f.s,
               (unsigned long)f.e, (unsigned long)row_a, (unsigned long)p);
        p = dummy;
      }
#endif
      asm volatile("" : "+v"(p));
      return reinterpret_cast<gptr_u32x4>(p);
    };
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    auto absorb = [&](u32x4 w, uint32_t r) {  // rows read from the pad are zero
      if ((r == rs0) | (r == rs1) | (r == re)) {
        const uint64_t a = row_a + (uint64_t)r * kRowBytes;
        w.x = frame_word(w.x, a, f.s, f.e, u);
        w.y = frame_word(w.y, a + 4, f.s, f.e, u);
        w.z = frame_word(w.z, a + 8, f.s, f.e, u);
        w.w = frame_word(w.w, a + 12, f.s, f.e, u);
      }
      if (r < rows) STEP_ROW(w);
    };
    // two banks of 4 rows, loads always issued (pad reads past the unit) so
    // that the loads in flight are counted exactly
    u32x4 ba[4], bb[4];
#pragma unroll
    for (uint32_t k2 = 0; k2 < 4; k2++) ba[k2] = __builtin_nontemporal_load(row_addr(k2));
    for (uint32_t r = 0; r < rows_max; r += 8) {
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) bb[k2] = __builtin_nontemporal_load(row_addr(r + 4 + k2));
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) absorb(ba[k2], r + k2);
      if (r + 4 >= rows_max) break;
      if (r + 8 < rows_max) {
#pragma unroll
        for (uint32_t k2 = 0; k2 < 4; k2++) ba[k2] = __builtin_nontemporal_load(row_addr(r + 8 + k2));
      }
#pragma unroll
      for (uint32_t k2 = 0; k2 < 4; k2++) absorb(bb[k2], r + 4 + k2);
    }
    const uint32_t raw = merge_braids(g_lds, c0, c1, c2, c3, lane_fin);
    if (active) {
      const uint32_t contrib = shift_units(g_lds, dc, raw, k);
#ifdef LSBM_DEBUG_BOUNDS
      if (li == 0 && b >= args.n) printf("ACC OOB wave %lu b %lu n %lu\n", (unsigned long)wave, (unsigned long)b, (unsigned long)args.n);
      else
#endif
      if (li == 0) atomicXor(args.acc + b, contrib);
    }
    // advance the cursor past the 8 units just taken
    const uint32_t pre8_prev = (uint32_t)__shfl((int)pre, (int)(jnext ? jnext - 1 : 0));
    const uint32_t pre8 = jnext ? pre8_prev : 0u;
    cur_b += jnext;
    cur_o = cur_o + 8 - pre8;
  }
}

// One thread per block: acc -> CRC -> output mode.
__global__ __launch_bounds__(256) void crc32c_finish_kernel(RaggedArgs args) {
  const DevConsts* __restrict__ dc = args.dc;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < args.n;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const Frame f = block_frame(args, b);
    const uint32_t z = (uint32_t)((f.row0 + f.rows) * kRowBytes - f.e);
#ifdef LSBM_DEBUG_BOUNDS
    if (z >= 128) { printf("Z OOB b %lu z %u s %lx e %lx row0 %lx rows %lu\n", (unsigned long)b, z, (unsigned long)f.s, (unsigned long)f.e, (unsigned long)f.row0, (unsigned long)f.rows); continue; }
#endif
    uint32_t l = nib_glb(dc->neg_nib[z], args.acc[b]);  // register after the block
    if (args.mode == kModeSstSeal) {
      const uint8_t typ = args.types[b];
      l = dc->t0[(l ^ typ) & 0xffu] ^ (l >> 8);  // Extend(crc, &type, 1)
    }
    const uint32_t crc = l ^ 0xffffffffu;
    switch (args.mode) {
      case kModeOut:
        args.out[b] = (args.flags & 1u) ? mask_crc(crc) : crc;
        break;
      case kModeVerify: {
        const uint32_t got = (args.flags & 1u) ? mask_crc(crc) : crc;
        const bool good = got == args.expect[b];
        args.ok[b] = good ? 1 : 0;
        if (!good && args.nbad) atomicAdd(args.nbad, 1u);
        break;
      }
      case kModeSstSeal: {  // table/table_builder.cc:245-249
        uint8_t* t = args.file + (f.e - reinterpret_cast<uint64_t>(args.base));
        const uint32_t m = mask_crc(crc);
        t[0] = args.types[b];
        t[1] = (uint8_t)m;
        t[2] = (uint8_t)(m >> 8);
        t[3] = (uint8_t)(m >> 16);
        t[4] = (uint8_t)(m >> 24);
        break;
      }
      default: {  // kModeSstVerify: table/format.cc:95-103
        const uint8_t* t = reinterpret_cast<const uint8_t*>(f.e);
        const uint32_t stored = (uint32_t)t[0] | ((uint32_t)t[1] << 8) |
                                ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
        const bool good = unmask_crc(stored) == crc;
        args.ok[b] = good ? 1 : 0;
        if (!good && args.nbad) atomicAdd(args.nbad, 1u);
        break;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Benchmark helpers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void fill_splitmix64_kernel(uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t seed) {
  const uint64_t nchunks = nbytes / 16;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t c = tid; c < nchunks; c += nthreads) {
    const uint64_t w0 = splitmix64(seed + 2 * c), w1 = splitmix64(seed + 2 * c + 1);
    reinterpret_cast<ulonglong2*>(buf)[c] = make_ulonglong2(w0, w1);
  }
  if (tid == 0) {
    for (uint64_t a = nchunks * 16; a < nbytes; a++)
      buf[a] = (uint8_t)(splitmix64(seed + (a >> 3)) >> (8 * (a & 7)));
  }
}

// Read ceiling for the CRC kernels' own access pattern: 1024-thread
// workgroups, each wave reads 8 blocks of 4 KiB as 128-B rows (one 16-B
// non-temporal load per lane per row), waves interleaved over 32 KiB groups;
// a grid-stride loop covers any remainder.  Bytes are xor-folded so the
// loads stay live.
__global__ __launch_bounds__(kBlockThreads) void stream_read_kernel(const uint8_t* __restrict__ base,
                                                                    uint64_t nbytes,
                                                                    uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63u, g = lane >> 3, li = lane & 7u;
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  const uint64_t ngroups = nbytes / 32768;
  uint32_t acc = 0;
  for (uint64_t grp = wave; grp < ngroups; grp += nwaves) {
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(base + grp * 32768), (short)0, 32768, 0x00020000);
    const uint32_t loff = g * 4096u + 16u * li;
#pragma unroll
    for (uint32_t r0 = 0; r0 < 32; r0 += 4) {
      u32x4 v[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; k++)
        v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsrc, loff + (r0 + k) * kRowBytes, 0, kAuxNT));
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) acc ^= xor3(v[k].x, v[k].y, v[k].z) ^ v[k].w;
    }
  }
  const uint64_t tail0 = ngroups * 32768;
  for (uint64_t i = tail0 + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i + 16 <= nbytes;
       i += (uint64_t)gridDim.x * blockDim.x * 16) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(base + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x & 1023u] = acc;  // keeps the loads live
}

// ---- host-callable launchers (C++ linkage, used by crc32c_engine.cc) ----
hipError_t launch_fixed(const uint8_t* base, uint64_t stride, uint32_t rows, uint64_t n_blocks,
                        const uint32_t* init, uint32_t* out, uint32_t flags, uint32_t k_value,
                        const DevConsts* dc, int grid, hipStream_t stream) {
#define LSBM_LAUNCH_FIXED(HI, R)                                                        \
  hipLaunchKernelGGL((crc32c_fixed_kernel<HI, R>), dim3(grid), dim3(kBlockThreads), 0, stream, \
                     base, stride, rows, n_blocks, init, out, flags, k_value, dc)
  // compile-time row counts for the SSTable-sized configs: 4 KiB and 64 KiB
  if (init) {
    if (rows == 32) LSBM_LAUNCH_FIXED(true, 32);
    else if (rows == 512) LSBM_LAUNCH_FIXED(true, 512);
    else LSBM_LAUNCH_FIXED(true, 0);
  } else {
    if (rows == 32) LSBM_LAUNCH_FIXED(false, 32);
    else if (rows == 512) LSBM_LAUNCH_FIXED(false, 512);
    else LSBM_LAUNCH_FIXED(false, 0);
  }
#undef LSBM_LAUNCH_FIXED
  return hipGetLastError();
}

// acc must hold n zeroed words.
hipError_t launch_ragged(const RaggedArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(crc32c_units_kernel, dim3(grid), dim3(kBlockThreads), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t fin_wgs = (a.n + 255) / 256;
  hipLaunchKernelGGL(crc32c_finish_kernel, dim3((unsigned)(fin_wgs < 65536 ? fin_wgs : 65536)),
                     dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(fill_splitmix64_kernel, dim3(grid), dim3(256), 0, stream, buf, nbytes, seed);
  return hipGetLastError();
}

hipError_t launch_stream_read(const void* buf, uint64_t nbytes, uint32_t* sink, int grid,
                              hipStream_t stream) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(kBlockThreads), 0, stream,
                     reinterpret_cast<const uint8_t*>(buf), nbytes, sink);
  return hipGetLastError();
}

}  // namespace lsbm
