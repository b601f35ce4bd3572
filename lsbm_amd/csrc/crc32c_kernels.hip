// crc32c_kernels.hip -- gfx950 kernels of the batched CRC-32C engine.
//
// crc32c_fixed_kernel   fixed-stride, len % 128 == 0, 16-B aligned blocks
//                       (SSTable-sized 4 KiB and 64 KiB batches; the headline)
// crc32c_units_kernel   any extents, any alignment (offsets[] batches, verify,
//                       SSTable trailer seal / verify, log headers): <= 48-row
//                       units per lane group, summed per block inside the wave
//                       and finished in registers
// fill_splitmix64_kernel, stream_read_kernel   benchmark helpers
//
// Both CRC kernels compute, per block, exactly what lsbm's
// crc32c::Extend(init, block, n) returns (util/crc32c.cc:286-329): the
// register starts at init ^ ~0 (:289), absorbs the bytes, and is inverted
// again (:328).  They differ from the reference only in how the bytes are
// absorbed (braids of A^128 steps instead of one serial A^4 chain).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "crc32c_units.h"

namespace lsbm {


#ifdef LSBM_DIAG_STAMPS  // diagnostic builds only: per-wave timeline (crc32c_units.h)
extern "C" __attribute__((visibility("default"))) int lsbm_diag_stamps(uint64_t* host, int n) {
  (void)n;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(uint64_t) * 4 * 65536) == hipSuccess ? 0 : -1;
}
#endif
#define DIAG_STAMP(k) DIAG_STAMP_W(k, wave)

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
    const DevConsts* __restrict__ dc, uint32_t* __restrict__ heads /* null: no cross-XCC queue */) {
  const uint32_t rows = kRows ? kRows : rows_arg;  // kRows != 0: fully unrolled
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = row_lane_base(lane);
  const uint32_t L0 = lb | kRowTab[0], L1 = lb | kRowTab[1], L2 = lb | kRowTab[2], L3 = lb | kRowTab[3];
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
  // Interleave: wave w starts at group w; a workgroup's k-th group is
  // (k / 16) * nwaves + 16 * blockIdx + k % 16, so at any moment the GPU
  // streams one contiguous window of the batch.  (A dynamic per-XCC work
  // queue in global memory was 5% slower end to end: DESIGN.md section 4.)
#ifndef LSBM_WG_STATIC
  // A workgroup's groups are the static interleave's, but its waves take them
  // in turn from an LDS counter, so a fast wave takes more of them: under the
  // static split the waves' durations spread with an 18% CV and the first wave
  // was done at 54% of the launch (tools/wave_spread.py);
  // with the counter, 3.8% and 87%.  (-DLSBM_WG_STATIC: the static split, A/B.)
  __shared__ uint32_t s_next;
  if (threadIdx.x == 0) s_next = kWavesPerWg;  // (ordered by load_lds_tables' barrier)
  auto next_grp = [&](uint64_t) -> uint64_t {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(&s_next, 1u);
    k = __builtin_amdgcn_readfirstlane(k);
#ifdef LSBM_WG_ROTATE  // A/B: row c of the interleave rotated by c workgroups
    const uint64_t c = k / kWavesPerWg;
    return c * nwaves + (((uint64_t)blockIdx.x + c) % gridDim.x) * kWavesPerWg + (k % kWavesPerWg);
#else
    return (uint64_t)(k / kWavesPerWg) * nwaves + (uint64_t)blockIdx.x * kWavesPerWg + (k % kWavesPerWg);
#endif
  };
#else
  auto next_grp = [&](uint64_t gp) -> uint64_t { return gp + nwaves; };
#endif
  // With the cross-XCC queue (crc32c_units.h): row 0 is the waves' own, the
  // rest comes in workgroup batches of W groups (items) from the heads.
  __shared__ uint32_t s_wq[kWqWords];
  const WgQueue<kWavesPerWg> wq{heads, (lds_u32*)s_wq,
                                ngroups > nwaves ? (ngroups - nwaves + kWavesPerWg - 1) / kWavesPerWg : 0};
  if (heads && threadIdx.x == 0) wq.init(xcc_id());  // (ordered by load_lds_tables' barrier)

  uint64_t grp = wave;
  DIAG_STAMP(0);
  bool loaded = false;  // the banks hold grp's first rows already
  if (grp < ngroups) {
    set_group(grp);
    LOAD_BANK(a, 0);
    if (kRows == 0 || kPF < rows) LOAD_BANK(b, kPF);
    loaded = true;
  }
  load_lds_tables(g_lds, dc);
  DIAG_STAMP(1);

  uint32_t pend_pub = heads && wave_in_wg == 0 ? kWqLead : 0u;  // a batch this wave publishes
  for (;;) {
    if (grp < ngroups) {
      const uint64_t blk = grp * 8 + g;
      const bool valid = blk < n_blocks;
      // Two banks of kPF rows: while one bank is absorbed the other's loads
      // are in flight.  Row 0 initialises the braids (c = w); every later row
      // is c = A^128(c) ^ w.
      if (!loaded) {
        set_group(grp);
        LOAD_BANK(a, 0);
        if (kRows == 0 || kPF < rows) LOAD_BANK(b, kPF);
      }
      loaded = false;
      if (pend_pub) {  // (behind this group's first loads: the claim's wait overlaps them)
        wq.publish(pend_pub);
        pend_pub = 0;
      }
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
    } else if (pend_pub) {
      wq.publish(pend_pub);
      pend_pub = 0;
    }
    if (!heads) {
      grp = next_grp(grp);
      if (grp >= ngroups) break;
      continue;
    }
    // the next slot: wave-group `slot` of batch `bt`
    const uint32_t k = wq.take(), bt = k / kWavesPerWg, slot = k % kWavesPerWg;
    if (slot == 0) pend_pub = bt + kWqLead;
    const uint32_t it = wq.read(bt);
    if (it == kWqNone) {
      if (pend_pub) wq.publish(pend_pub);  // (kWqNone as well; no wave of this workgroup waits for it)
      break;
    }
    grp = nwaves + (uint64_t)it * kWavesPerWg + slot;  // (past ngroups in the last item: a slot without a group)
  }
  DIAG_STAMP(2);
  DIAG_XCC_W(wave);
}
// ---------------------------------------------------------------------------
// Ragged path (crc32c_units.h): the units kernel walks each wave's range of
// blocks in rounds of 8 units.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// Trailer scatter: the second pass of lsbm_sst_seal_dev.  The units kernel
// computes the CRCs densely (SstCrc mode); this pass merges trailer i =
// [types[i]][crc LE32] into file[off + size, +5) for every handle that fits.
// Each merge is a compare-and-swap on the aligned 8-byte word(s) covering the
// bytes (correct when records shorter than 11 bytes share a word).  Measured
// on 1M x 4,118-B blocks: the scattered 5-byte writes cost the read-streaming
// kernel 13 points of HBM bandwidth when done in it, and a separate pass of
// byte stores as much again (0.17 ms); the compare-and-swap pass, ~0.03 ms.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cas_merge(unsigned long long* p, uint64_t m, uint64_t v) {
  unsigned long long old = *p;
  for (;;) {
    const unsigned long long want = (old & ~m) | (v & m);
    if (want == old) return;
    const unsigned long long got = atomicCAS(p, old, want);
    if (got == old) return;
    old = got;
  }
}

// nb (<= 5) little-endian bytes of v at address t of the image [img, img + limit)
__device__ __forceinline__ void merge_bytes(uint64_t img, uint64_t limit, uint64_t t, uint32_t nb, uint64_t v) {
  const uint32_t sh = (uint32_t)(t & 7u);
  const uint64_t w0a = t & ~7ull;
  const bool two = sh + nb > 8;
  if (w0a < img || w0a + (two ? 16u : 8u) > img + limit) {  // words reaching outside: bytes
    uint8_t* tb = reinterpret_cast<uint8_t*>(t);
    for (uint32_t k = 0; k < nb; k++) tb[k] = (uint8_t)(v >> (8 * k));
    return;
  }
  const uint64_t fm = (1ull << (8 * nb)) - 1;
  unsigned long long* w = reinterpret_cast<unsigned long long*>(w0a);
  cas_merge(w, fm << (8 * sh), v << (8 * sh));
  if (two) cas_merge(w + 1, fm >> (64 - 8 * sh), v >> (64 - 8 * sh));
}

__global__ __launch_bounds__(256) void trailer_scatter_kernel(uint8_t* __restrict__ file, uint64_t limit,
                                                              const uint64_t* __restrict__ handles,
                                                              const uint8_t* __restrict__ types,
                                                              const uint32_t* __restrict__ crcs, uint64_t n) {
  const uint64_t img = reinterpret_cast<uint64_t>(file);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t off = handles[2 * i], size = handles[2 * i + 1];
    if (!(off <= limit && limit - off >= kTrailer && limit - off - kTrailer >= size)) continue;
    merge_bytes(img, limit, img + off + size, 5, (uint64_t)types[i] | ((uint64_t)crcs[i] << 8));
  }
}

// The units kernel; in SstCrc mode with args.file set (lsbm_sst_seal_dev) each
// wave then merges the trailers of its own blocks into the image, from the
// dense CRCs it has just written: the seal's trailer writes happen after the
// wave's last row load (none of them queues in front of its reads) and
// overlap the other waves' streaming, instead of a second pass over the
// trailers after the kernel.
// kPieces (launch_ragged: a chunked sweep, or SSTable trailer pieces): the
// walk over pieces; otherwise the walk of one range, compiled without the
// piece code.  Two kernels rather than two walks in one: with both inlined
// the one-range walks (the fused seal's among them) ran 1.3-2 points slower
// than round 5's single-walk kernel on the same box (profiles/r06/events_ab/).
template <uint32_t kMaxRows, uint32_t kMode, uint32_t kExt, bool kPieces>
__global__ __launch_bounds__(kBlockThreads) void crc32c_units_kernel(RaggedArgs args) {
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  bool chunked;
  uint32_t pi, p_end;
  uint64_t b_lo, b_hi;
  DIAG_STAMP(0);
  wave_range<kMode, kExt>(args, wave, nwaves, chunked, pi, p_end, b_lo, b_hi);
  DIAG_STAMP(1);
  if constexpr (kPieces) {
#ifndef LSBM_PIECES_STATIC
    // the pieces are claimed from an LDS counter (next_piece); the walk claims
    // before its table fill's barrier, hence one of its own
    __shared__ uint32_t s_claim;
    if (threadIdx.x == 0) s_claim = kWavesPerWg;
    __syncthreads();
    units_walk<kMaxRows, kMode, kExt, true>(args, wave, nwaves, b_lo, b_hi, chunked, pi, p_end, true, 0,
                                            (lds_u32*)&s_claim);
#else
    units_walk<kMaxRows, kMode, kExt>(args, wave, nwaves, b_lo, b_hi, chunked, pi, p_end, true);
#endif
  } else {
    units_walk<kMaxRows, kMode, kExt, false, kWavesPerWg, false>(args, wave, nwaves, b_lo, b_hi, false, pi, p_end,
                                                                true);
  }
  if constexpr (kMode == kModeSstCrc && kExt == kExtHandles) {
    if (args.file != nullptr) {  // (SstCrc is never chunked: [b_lo, b_hi) is this wave's range)
      // this wave's out[] stores complete (s_waitcnt vmcnt(0)) before it reads
      // them back past L1 (an agent-scope fence would write back the whole L2)
      __builtin_amdgcn_s_waitcnt(0x0F70);
      const uint64_t img = reinterpret_cast<uint64_t>(args.file), limit = args.limit;
      const uint32_t lane = threadIdx.x & 63u;
      for (uint64_t i = b_lo + lane; i < b_hi; i += 64) {
        const uint64_t off = args.handles[2 * i], size = args.handles[2 * i + 1];
        if (!(off <= limit && limit - off >= kTrailer && limit - off - kTrailer >= size)) continue;
        const uint32_t crc = __hip_atomic_load(args.out + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        merge_bytes(img, limit, img + off + size, 5, (uint64_t)args.types[i] | ((uint64_t)crc << 8));
      }
    }
  }
  DIAG_STAMP(2);
  DIAG_XCC_W(wave);
}

// ---------------------------------------------------------------------------
// Gather: dst[dst_off[i], +len[i]) = src[src_off[i], +len[i]), one wave per
// segment (grid-stride), 16-B stores where both sides allow, bytes elsewhere.
// Compacts variable-length outputs before they go back to the host
// (block_compression.cc: only the compressed bytes, not their capacity slots).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* __restrict__ src,
                                                     const uint64_t* __restrict__ src_off,
                                                     const uint64_t* __restrict__ len, uint64_t n,
                                                     uint8_t* __restrict__ dst,
                                                     const uint64_t* __restrict__ dst_off) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t i = wave; i < n; i += nwaves) {
    const uint8_t* a = src + src_off[i];
    uint8_t* b = dst + dst_off[i];
    const uint64_t m = len[i];
    if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) == 0) {
      const uint64_t m16 = m / 16;
      for (uint64_t k = lane; k < m16; k += 64)
        reinterpret_cast<u32x4*>(b)[k] = reinterpret_cast<const u32x4*>(a)[k];
      for (uint64_t k = m16 * 16 + lane; k < m; k += 64) b[k] = a[k];
    } else {
      for (uint64_t k = lane; k < m; k += 64) b[k] = a[k];
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
                        const DevConsts* dc, int grid, hipStream_t stream, uint32_t* heads) {
#define LSBM_LAUNCH_FIXED(HI, R)                                                        \
  hipLaunchKernelGGL((crc32c_fixed_kernel<HI, R>), dim3(grid), dim3(kBlockThreads), 0, stream, \
                     base, stride, rows, n_blocks, init, out, flags, k_value, dc, heads)
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

hipError_t launch_range_bounds(const RaggedArgs& a, uint64_t P, uint32_t* bounds, int grid,
                               hipStream_t stream) {
  const uint64_t want = (P / 2 + 1 + 3) / 4;  // 4 waves per workgroup, two bounds per wave
  const dim3 g((unsigned)(want < (uint64_t)grid ? want : grid));
  if (a.extents == kExtOffsets)
    hipLaunchKernelGGL(range_bounds_kernel<kExtOffsets>, g, dim3(256), 0, stream, a, P, bounds);
  else if (a.extents == kExtHandles)
    hipLaunchKernelGGL(range_bounds_kernel<kExtHandles>, g, dim3(256), 0, stream, a, P, bounds);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// crc32c_stream.hip
bool stream_eligible(const RaggedArgs& a);
hipError_t launch_stream(const RaggedArgs& a, int grid, hipStream_t stream);

// Which kernel a ragged batch runs on: batches of offsets[], SSTable handles
// and log headers with no per-block init stream their rows
// (crc32c_stream_kernel; extents out of order just make shorter sub-pieces).
// LSBM_RAGGED_KERNEL=units keeps every batch on the units kernel (A/B runs).
// Which ragged kernel a batch runs on.  The stream kernel wins on offsets[]
// batches of mixed block sizes (config 4: 78-80 vs 75-76 % of HBM peak) and
// on log images (WAL records of 0-2,540 B: 45-53 vs 44-48 %) and loses on
// SSTable images (4 KiB blocks between trailers: 74-77 vs 78-82 %; DESIGN.md
// section 4), so by default offsets[] batches and log headers take it.
// LSBM_RAGGED_KERNEL=units | stream (or lsbm_test_ragged_kernel) overrides:
// every batch on the units kernel, or every eligible one on the stream kernel.
namespace {
std::atomic<int> g_ragged_policy{-1};  // -1: not read yet; 0 default, 1 units, 2 stream
int ragged_policy() {
  int p = g_ragged_policy.load(std::memory_order_relaxed);
  if (p < 0) {
    const char* v = getenv("LSBM_RAGGED_KERNEL");
    p = v && v[0] == 'u' ? 1 : (v && v[0] == 's' ? 2 : 0);
    int expect = -1;
    if (!g_ragged_policy.compare_exchange_strong(expect, p)) p = expect;
  }
  return p;
}
}  // namespace

bool ragged_uses_stream(const RaggedArgs& a) {
  const int p = ragged_policy();
  if (p == 1 || !stream_eligible(a)) return false;
  return p == 2 || a.extents == kExtOffsets || a.extents == kExtLogHeaders;
}

int set_ragged_policy(int p) {
  if (p < 0 || p > 2) return -1;
  g_ragged_policy.store(p);
  return 0;
}

// The units kernel for a's schedule: over pieces when the engine set a chunked
// sweep (bounds) or SSTable trailer pieces (nchunks), wave_range's `chunked`.
template <uint32_t R, uint32_t M, uint32_t X>
void launch_units(const RaggedArgs& a, int grid, hipStream_t stream) {
  if constexpr (kCanChunk<M, X>) {
    if (a.bounds != nullptr || a.nchunks != 0) {
      hipLaunchKernelGGL((crc32c_units_kernel<R, M, X, true>), dim3(grid), dim3(kBlockThreads), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((crc32c_units_kernel<R, M, X, false>), dim3(grid), dim3(kBlockThreads), 0, stream, a);
}

// grid: one workgroup per CU (the LDS image); the waves per workgroup differ
// (kWavesPerWg, kStreamWavesPerWg), and a chunked sweep's bounds (a.bounds)
// must have been computed for the kernel's wave count.
hipError_t launch_ragged(const RaggedArgs& a, int grid, hipStream_t stream) {
  if (ragged_uses_stream(a)) return launch_stream(a, grid, stream);
#define LSBM_LAUNCH_UNITS(R, M, X) launch_units<R, M, X>(a, grid, stream)
  switch (a.mode) {
    case kModeOut:
      if (a.extents == kExtOffsets) LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeOut, kExtOffsets);
      else if (a.extents == kExtHandles) LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeOut, kExtHandles);
      else if (a.extents == kExtFixed) LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeOut, kExtFixed);
      else return hipErrorInvalidValue;
      break;
    case kModeVerify:
      if (a.extents != kExtOffsets) return hipErrorInvalidValue;
      LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeVerify, kExtOffsets);
      break;
    case kModeSstSeal:
      LSBM_LAUNCH_UNITS(kSstUnitRows, kModeSstSeal, kExtHandles);
      break;
    case kModeSstVerify:
      LSBM_LAUNCH_UNITS(kSstUnitRows, kModeSstVerify, kExtHandles);
      break;
    case kModeSstCrc:
      LSBM_LAUNCH_UNITS(kSstUnitRows, kModeSstCrc, kExtHandles);
      break;
    case kModeLogSeal:
      LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeLogSeal, kExtLogHeaders);
      break;
    case kModeLogVerify:
      LSBM_LAUNCH_UNITS(LSBM_UNIT_ROWS, kModeLogVerify, kExtLogHeaders);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef LSBM_LAUNCH_UNITS
  return hipGetLastError();
}

hipError_t launch_trailer_scatter(uint8_t* file, uint64_t limit, const uint64_t* handles, const uint8_t* types,
                                  const uint32_t* crcs, uint64_t n, int grid, hipStream_t stream) {
  const uint64_t want = (n + 255) / 256;
  hipLaunchKernelGGL(trailer_scatter_kernel, dim3((unsigned)(want < (uint64_t)grid ? want : grid)), dim3(256), 0,
                     stream, file, limit, handles, types, crcs, n);
  return hipGetLastError();
}

hipError_t launch_gather(const uint8_t* src, const uint64_t* src_off, const uint64_t* len, uint64_t n,
                         uint8_t* dst, const uint64_t* dst_off, int grid, hipStream_t stream) {
  const uint64_t want = (n + 3) / 4;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)(want < (uint64_t)grid ? want : grid)), dim3(256), 0,
                     stream, src, src_off, len, n, dst, dst_off);
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
