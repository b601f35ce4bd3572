// crc32c_kernels.hip -- gfx950 kernels of the batched CRC-32C engine.
//
// crc32c_fixed_kernel   fixed-stride, len % 128 == 0, 16-B aligned blocks
//                       (SSTable-sized 4 KiB and 64 KiB batches; the headline)
// crc32c_ragged_kernel  any extents, any alignment: offsets[] batches, verify,
//                       and the SSTable trailer seal / verify modes
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

constexpr uint32_t kPF = 4;  // rows per load bank

// Issue the loads of rows [r0, r0 + kPF) of this lane's slice into bank X.
// Always kPF loads (rows past the end re-read the last row, a cache hit) so
// that the compiler can count outstanding loads exactly; `rows` is uniform.
#define LOAD_BANK(X, r0)                                                        \
  do {                                                                          \
    _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPF; k_++) {                   \
      const uint32_t rr_ = (r0) + k_ < rows ? (r0) + k_ : rows - 1;             \
      X[k_] = __builtin_nontemporal_load(p + rr_ * 8);                          \
    }                                                                           \
  } while (0)

#define STEP_ROW(W)                                          \
  do {                                                       \
    s0 = row_step(g_lds, s0 ^ (W).x, L0, L1, L2, L3);        \
    s1 = row_step(g_lds, s1 ^ (W).y, L0, L1, L2, L3);        \
    s2 = row_step(g_lds, s2 ^ (W).z, L0, L1, L2, L3);        \
    s3 = row_step(g_lds, s3 ^ (W).w, L0, L1, L2, L3);        \
  } while (0)

// All kPF rows of the bank are followed by more rows: advance by 128 B each.
#define ABSORB_FULL(X)                                              \
  do {                                                              \
    _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPF; k_++) STEP_ROW(X[k_]); \
  } while (0)

// The bank holds the block's last row: rows before it advance, the last row
// is only xor-ed in (its registers are merged by merge_braids).
#define ABSORB_TAIL(X, r0)                                    \
  do {                                                        \
    _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPF; k_++) { \
      if ((r0) + k_ + 1 < rows) {                             \
        STEP_ROW(X[k_]);                                      \
      } else if ((r0) + k_ + 1 == rows) {                     \
        s0 ^= X[k_].x;                                        \
        s1 ^= X[k_].y;                                        \
        s2 ^= X[k_].z;                                        \
        s3 ^= X[k_].w;                                        \
      }                                                       \
    }                                                         \
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
  load_lds_tables(g_lds, dc);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = (lane & 31u) << 2;
  const uint32_t L0 = lb, L1 = lb | 0x80u, L2 = lb | 0x10000u, L3 = lb | 0x10080u;
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  const uint64_t ngroups = (n_blocks + 7) / 8;

  for (uint64_t grp = wave; grp < ngroups; grp += nwaves) {
    const uint64_t blk = grp * 8 + g;
    const bool valid = blk < n_blocks;
    const u32x4* __restrict__ p =
        reinterpret_cast<const u32x4*>(base + (valid ? blk : 0) * stride) + li;
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;

    // Two banks of kPF rows each: while bank A is absorbed, bank B's loads
    // are in flight (and vice versa), so every lane keeps kPF..2*kPF rows of
    // 16 B outstanding without the compiler rotating registers.
    u32x4 a[kPF], b[kPF];
    LOAD_BANK(a, 0);
    uint32_t r = 0;
    // steady state: both banks hold rows that are followed by more rows
    while (r + 3 * kPF <= rows) {
      LOAD_BANK(b, r + kPF);
      ABSORB_FULL(a);
      LOAD_BANK(a, r + 2 * kPF);
      ABSORB_FULL(b);
      r += 2 * kPF;
    }
    // the last (up to 3) banks
    while (true) {
      if (r + kPF < rows) {
        LOAD_BANK(b, r + kPF);
        ABSORB_FULL(a);
      } else {
        ABSORB_TAIL(a, r);
        break;
      }
      r += kPF;
      if (r + kPF < rows) {
        LOAD_BANK(a, r + kPF);
        ABSORB_FULL(b);
      } else {
        ABSORB_TAIL(b, r);
        break;
      }
      r += kPF;
    }
    const uint32_t raw = merge_braids(g_lds, s0, s1, s2, s3, li);
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
}

// ---------------------------------------------------------------------------
// Ragged kernel.  Same row/braid machinery, but rows are 128-B aligned in the
// absolute address space, so every load is an aligned 16-B load whatever the
// block's alignment.  For block [s, e):
//   * bytes of the frame outside [s, e) are zero; leading zeros leave a raw
//     CRC unchanged, so the frame may start early for free;
//   * the init register v = init ^ ~0 is injected as 4 virtual bytes
//     u = A^-4(v) at [s-4, s) (absorbing u from zero gives exactly v);
//   * the frame ends z = frame_end - e bytes late: undone with A^-z.
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

__global__ __launch_bounds__(kBlockThreads) void crc32c_ragged_kernel(RaggedArgs args) {
  const DevConsts* __restrict__ dc = args.dc;
  load_lds_tables(g_lds, dc);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = (lane & 31u) << 2;
  const uint32_t L0 = lb, L1 = lb | 0x80u, L2 = lb | 0x10000u, L3 = lb | 0x10080u;
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerWg + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerWg;
  const uint64_t ngroups = (args.n + 7) / 8;
  const uint64_t base_addr = reinterpret_cast<uint64_t>(args.base);

  for (uint64_t grp = wave; grp < ngroups; grp += nwaves) {
    const uint64_t blk = grp * 8 + g;
    const bool valid = blk < args.n;
    uint64_t s = base_addr, e = base_addr;
    if (valid) {
      if (args.extents == kExtHandles) {
        const uint64_t off = args.handles[2 * blk], sz = args.handles[2 * blk + 1];
        s = base_addr + off;
        e = s + sz + (args.mode == kModeSstVerify ? 1u : 0u);  // verify covers the type byte
      } else if (args.extents == kExtFixed) {
        s = base_addr + blk * args.stride;
        e = s + args.len;
      } else {
        s = base_addr + args.offsets[blk];
        e = base_addr + args.offsets[blk + 1];
        if (e < s) e = s;
      }
    }
    const uint32_t v = (args.init && valid ? args.init[blk] : 0u) ^ 0xffffffffu;
    const uint32_t u = nib_glb(dc->neg4_nib, v);
    const uint64_t row0 = (s - 4) >> 7;
    const uint64_t row_end = (e + 127) >> 7;  // one past the last row
    const uint64_t rows = row_end > row0 ? row_end - row0 : 1;
    const uint32_t z = (uint32_t)((row0 + rows) * kRowBytes - e);

    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (uint64_t r = 0; r < rows; r++) {
      const uint64_t a = (row0 + r) * kRowBytes + 16u * li;
      u32x4 w = {0u, 0u, 0u, 0u};
      if (a + 16 > s - 4 && a < e) {
        if (s < e && a + 16 > s && a < e) w = *reinterpret_cast<const u32x4*>(a);
        if (a < s || a + 16 > e) {
          w.x = frame_word(w.x, a, s, e, u);
          w.y = frame_word(w.y, a + 4, s, e, u);
          w.z = frame_word(w.z, a + 8, s, e, u);
          w.w = frame_word(w.w, a + 12, s, e, u);
        }
      }
      if (r + 1 < rows) {
        s0 = row_step(g_lds, s0 ^ w.x, L0, L1, L2, L3);
        s1 = row_step(g_lds, s1 ^ w.y, L0, L1, L2, L3);
        s2 = row_step(g_lds, s2 ^ w.z, L0, L1, L2, L3);
        s3 = row_step(g_lds, s3 ^ w.w, L0, L1, L2, L3);
      } else {
        s0 ^= w.x;
        s1 ^= w.y;
        s2 ^= w.z;
        s3 ^= w.w;
      }
    }
    const uint32_t padded = merge_braids(g_lds, s0, s1, s2, s3, li);
    if (li == 7u && valid) {
      uint32_t l = nib_glb(dc->neg_nib[z], padded);  // register after the block
      if (args.mode == kModeSstSeal) {
        const uint8_t typ = args.types[blk];
        l = dc->t0[(l ^ typ) & 0xffu] ^ (l >> 8);  // Extend(crc, &type, 1)
      }
      const uint32_t crc = l ^ 0xffffffffu;
      switch (args.mode) {
        case kModeOut:
          args.out[blk] = (args.flags & 1u) ? mask_crc(crc) : crc;
          break;
        case kModeVerify: {
          const uint32_t got = (args.flags & 1u) ? mask_crc(crc) : crc;
          const bool good = got == args.expect[blk];
          args.ok[blk] = good ? 1 : 0;
          if (!good && args.nbad) atomicAdd(args.nbad, 1u);
          break;
        }
        case kModeSstSeal: {
          uint8_t* t = args.file + (e - base_addr);
          const uint32_t m = mask_crc(crc);
          t[0] = args.types[blk];
          t[1] = (uint8_t)m;
          t[2] = (uint8_t)(m >> 8);
          t[3] = (uint8_t)(m >> 16);
          t[4] = (uint8_t)(m >> 24);
          break;
        }
        default: {  // kModeSstVerify: table/format.cc:95-103
          const uint8_t* t = reinterpret_cast<const uint8_t*>(e);
          const uint32_t stored = (uint32_t)t[0] | ((uint32_t)t[1] << 8) |
                                  ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
          const bool good = unmask_crc(stored) == crc;
          args.ok[blk] = good ? 1 : 0;
          if (!good && args.nbad) atomicAdd(args.nbad, 1u);
          break;
        }
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

__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                          uint32_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = tid;
  for (; i + 3 * nthreads < n16; i += 4 * nthreads) {
    const u32x4 a = __builtin_nontemporal_load(p + i);
    const u32x4 b = __builtin_nontemporal_load(p + i + nthreads);
    const u32x4 c = __builtin_nontemporal_load(p + i + 2 * nthreads);
    const u32x4 d = __builtin_nontemporal_load(p + i + 3 * nthreads);
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^
           d.z ^ d.w;
  }
  for (; i < n16; i += nthreads) {
    const u32x4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
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
  if (init) {
    if (rows == 32) LSBM_LAUNCH_FIXED(true, 32);
    else LSBM_LAUNCH_FIXED(true, 0);
  } else {
    if (rows == 32) LSBM_LAUNCH_FIXED(false, 32);  // 4 KiB blocks: the headline config
    else LSBM_LAUNCH_FIXED(false, 0);
  }
#undef LSBM_LAUNCH_FIXED
  return hipGetLastError();
}

hipError_t launch_ragged(const RaggedArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(crc32c_ragged_kernel, dim3(grid), dim3(kBlockThreads), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(fill_splitmix64_kernel, dim3(grid), dim3(256), 0, stream, buf, nbytes, seed);
  return hipGetLastError();
}

hipError_t launch_stream_read(const void* buf, uint64_t nbytes, uint32_t* sink, int grid,
                              hipStream_t stream) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4*>(buf), nbytes / 16, sink);
  return hipGetLastError();
}

}  // namespace lsbm
