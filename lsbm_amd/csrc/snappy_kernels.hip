// snappy_kernels.hip -- batched snappy raw-format codec for gfx950: the
// SSTable block compression of TableBuilder::WriteBlock
// (table/table_builder.cc:181-193 -> port::Snappy_Compress -> snappy::RawCompress)
// and its inverse in ReadBlock (table/format.cc:124-141 ->
// Snappy_GetUncompressedLength / Snappy_Uncompress).  Byte-exact with the
// libsnappy the oracle is pinned to (oracle/snappy_oracle.c).
//
// A snappy stream is a chain of tags, each found only by parsing the previous
// one, so a block is one wave's serial work:
//  * the tag walk is wave-uniform (values broadcast with readfirstlane, so the
//    branches are scalar), and each literal / copy is spread over the 64 lanes;
//  * the wave's LDS slice holds the block: the decoder stages the compressed
//    bytes and decodes into an LDS output window, then writes the window out
//    coalesced; the encoder stages the fragment and keeps the uint16 hash
//    table beside it, and extends matches 64 bytes per step with a ballot;
//  * a block too large for the slice runs the same code against global
//    memory (template flag kLds = false).
// Throughput comes from many blocks in flight: one wave per workgroup, as many
// workgroups as LDS allows (snappy_types.h), grid-stride over the batch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "snappy_types.h"

namespace lsbm {
namespace {

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

// Orders the wave's own memory phases: its LDS (and, for the global-memory
// variant, its global) writes are complete and visible to every lane before
// the next access, and the compiler does not move accesses across.
__device__ __forceinline__ void wave_phase() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

// 8 bytes from p[i] on: LDS reads are two aligned dwords (the staged copy is
// padded, so this never reads past the slice); global reads are bytes bounded
// by n (zero past the end).
template <bool kLds>
__device__ __forceinline__ uint64_t load8(const uint8_t* p, uint32_t i, uint32_t n) {
  if (kLds) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (i & ~3u));
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return v >> (8 * (i & 3u));
  } else {
    uint64_t v = 0;
    for (uint32_t k = 0; k < 5; k++)
      if (i + k < n) v |= (uint64_t)p[i + k] << (8 * k);
    return v;
  }
}

template <bool kLds>
__device__ __forceinline__ uint32_t load32(const uint8_t* p, uint32_t i) {
  if (kLds) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (i & ~3u));
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return (uint32_t)(v >> (8 * (i & 3u)));
  } else {
    return (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) |
           ((uint32_t)p[i + 3] << 24);
  }
}

// snappy::GetUncompressedLength (varint32, <= 5 bytes, 5th < 16).
// Returns the preamble size, 0 on failure.
__device__ __forceinline__ uint32_t parse_preamble(const uint8_t* p, uint64_t n, uint32_t* ulen) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < 5; i++) {
    if (i >= n) return 0;
    const uint32_t b = p[i];
    if (i == 4 && b >= 16) return 0;
    v |= (b & 127u) << (7 * i);
    if (b < 128) {
      *ulen = v;
      return i + 1;
    }
  }
  return 0;
}

// ---- decoder ----

// Tag walk of snappy's DecompressAllTags over in[0, cl) into out[0, ulen):
// false on any condition RawUncompress rejects (oracle/snappy_oracle.c
// so_uncompress lists them).  Wave-uniform control flow.
template <bool kLds>
__device__ bool decode(const uint8_t* in, uint32_t cl, uint8_t* out, uint32_t ulen, uint32_t lane) {
  uint32_t ip = 0, op = 0;
  uint32_t fenced = 0;  // global variant: out[0, fenced) is visible to every lane
  while (ip < cl) {
    const uint64_t w = uni64(load8<kLds>(in, ip, cl));
    const uint32_t c = (uint32_t)w & 0xffu;
    if ((c & 3u) == 0) {  // literal
      uint64_t len = (c >> 2) + 1;
      uint32_t hdr = 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60;
        if (nb > cl - ip - 1) return false;
        const uint64_t m = nb == 4 ? 0xffffffffull : ((1ull << (8 * nb)) - 1);
        len = ((w >> 8) & m) + 1;
        hdr += nb;
      }
      if (len > (uint64_t)(cl - ip - hdr) || len > (uint64_t)(ulen - op)) return false;
      const uint8_t* src = in + ip + hdr;
      uint8_t* dst = out + op;
      for (uint32_t j = lane; j < (uint32_t)len; j += 64) dst[j] = src[j];
      ip += hdr + (uint32_t)len;
      op += (uint32_t)len;
    } else {  // copy
      uint32_t hdr, len, off;
      const uint32_t kind = c & 3u;
      if (kind == 1) {
        hdr = 2;
        len = 4 + ((c >> 2) & 7u);
        off = ((c >> 5) << 8) | (uint32_t)((w >> 8) & 0xffu);
      } else if (kind == 2) {
        hdr = 3;
        len = (c >> 2) + 1;
        off = (uint32_t)((w >> 8) & 0xffffu);
      } else {
        hdr = 5;
        len = (c >> 2) + 1;
        off = (uint32_t)((w >> 8) & 0xffffffffu);
      }
      if (hdr > cl - ip || off == 0 || off > op || len > ulen - op) return false;
      if (!kLds && op - off + (off < len ? off : len) > fenced) {
        wave_phase();
        fenced = op;
      }
      // byte j of the copy is out[op - off + j mod off]: an overlapping copy
      // (off < len) repeats its first off bytes, all written before it.
      if (lane < len) {
        const uint32_t k = off >= len ? lane : lane % off;
        out[op + lane] = out[op - off + k];
      }
      ip += hdr;
      op += len;
    }
    if (kLds) wave_phase();
  }
  return op == ulen;
}

__global__ __launch_bounds__(kSnapThreads) void snappy_uncompress_kernel(SnapDecArgs a) {
  const uint32_t lane = threadIdx.x;
  uint8_t* const lds_in = smem;
  for (uint64_t b = blockIdx.x; b < a.n; b += gridDim.x) {
    const uint64_t s = a.offsets[b], e = a.offsets[b + 1];
    const uint64_t os = a.out_offsets[b], cap = a.out_offsets[b + 1] - os;
    const uint64_t clen = e - s;
    uint32_t ulen = 0;
    const uint32_t pre = uni(parse_preamble(a.base + s, clen, &ulen));
    ulen = uni(ulen);
    bool ok = pre != 0 && (uint64_t)ulen <= cap;
    if (ok) {
      const uint64_t cl64 = clen - pre;
      const uint32_t cl_pad = (uint32_t)((cl64 + 8 + 15) & ~15ull);
      if (cl64 + 8 + 15 + (uint64_t)ulen <= kSnapDecLds) {
        const uint8_t* g = a.base + s + pre;
        const uint32_t cl = (uint32_t)cl64;
        for (uint32_t j = lane; j < cl + 8; j += 64) lds_in[j] = j < cl ? g[j] : 0;
        uint8_t* win = smem + cl_pad;
        wave_phase();
        ok = decode<true>(lds_in, cl, win, ulen, lane);
        if (ok) {
          uint8_t* dst = a.out + os;
          for (uint32_t j = lane; j < ulen; j += 64) dst[j] = win[j];
        }
        wave_phase();
      } else if (cl64 < 0xffffffffull) {
        ok = decode<false>(a.base + s + pre, (uint32_t)cl64, a.out + os, ulen, lane);
      } else {
        ok = false;  // a >= 4 GiB compressed block (snappy's lengths are 32-bit)
      }
    }
    if (lane == 0) {
      a.ok[b] = ok ? 1 : 0;
      if (!ok && a.n_bad) atomicAdd(a.n_bad, 1u);
    }
  }
}

__global__ __launch_bounds__(256) void snappy_length_kernel(SnapLenArgs a) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < a.n;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = a.offsets[b];
    uint32_t ulen = 0;
    const uint32_t pre = parse_preamble(a.base + s, a.offsets[b + 1] - s, &ulen);
    a.ulen[b] = pre ? ulen : 0;
    a.ok[b] = pre ? 1 : 0;
  }
}

// ---- encoder ----

__device__ __forceinline__ uint32_t table_size_for(uint32_t n) {
  if (n > kSnapMaxTable) return kSnapMaxTable;
  uint32_t t = 256;
  while (t < n) t <<= 1;
  return t;
}

__device__ __forceinline__ uint32_t hash_bytes(uint32_t bytes, uint32_t mask) {
  return ((bytes * 0x1e35a7bdu) >> (32 - kSnapMaxTableBits)) & mask;
}

// out[op..] = literal tag + in[0, len); returns the new op.
__device__ __forceinline__ uint64_t emit_literal(uint8_t* out, uint64_t op, const uint8_t* lit,
                                                 uint32_t len, uint32_t lane) {
  const uint32_t n = len - 1;
  uint32_t hdr = 1;
  if (n < 60) {
    if (lane == 0) out[op] = (uint8_t)(n << 2);
  } else {
    const uint32_t count = n < 256 ? 1 : n < 65536 ? 2 : n < (1u << 24) ? 3 : 4;
    if (lane == 0) out[op] = (uint8_t)((59 + count) << 2);
    if (lane >= 1 && lane <= count) out[op + lane] = (uint8_t)(n >> (8 * (lane - 1)));
    hdr += count;
  }
  uint8_t* dst = out + op + hdr;
  for (uint32_t j = lane; j < len; j += 64) dst[j] = lit[j];
  return op + hdr + len;
}

__device__ __forceinline__ uint64_t emit_copy_le64(uint8_t* out, uint64_t op, uint32_t off,
                                                   uint32_t len, bool lt12, uint32_t lane) {
  if (lt12 && off < 2048) {
    if (lane == 0) out[op] = (uint8_t)(1u + ((len - 4) << 2) + ((off >> 3) & 0xe0u));
    if (lane == 1) out[op + 1] = (uint8_t)off;
    return op + 2;
  }
  if (lane == 0) out[op] = (uint8_t)(2u + ((len - 1) << 2));
  if (lane == 1) out[op + 1] = (uint8_t)off;
  if (lane == 2) out[op + 2] = (uint8_t)(off >> 8);
  return op + 3;
}

__device__ __forceinline__ uint64_t emit_copy(uint8_t* out, uint64_t op, uint32_t off, uint32_t len,
                                              uint32_t lane) {
  if (len < 12) return emit_copy_le64(out, op, off, len, true, lane);
  while (len >= 68) {
    op = emit_copy_le64(out, op, off, 64, false, lane);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_le64(out, op, off, 60, false, lane);
    len -= 60;
  }
  return emit_copy_le64(out, op, off, len, len < 12, lane);
}

// Bytes matching from s1 = in[a], s2 = in[b] (a < b), up to in[end): 64 per
// step, first mismatch by ballot.
__device__ __forceinline__ uint32_t match_len(const uint8_t* in, uint32_t a, uint32_t b,
                                              uint32_t end, uint32_t lane) {
  uint32_t m = 0;
  for (;;) {
    const uint32_t rem = end - (b + m);
    const bool stop = lane >= rem || in[a + m + (lane < rem ? lane : 0)] != in[b + m + (lane < rem ? lane : 0)];
    const uint64_t mask = __ballot(stop);
    if (mask) return m + (uint32_t)__builtin_ctzll(mask);
    m += 64;
  }
}

// snappy.cc CompressFragment over in[0, n) (n <= 64 KiB) with a zeroed table
// of tsize entries; the walk mirrors oracle/snappy_oracle.c compress_fragment.
template <bool kLds>
__device__ uint64_t compress_fragment(const uint8_t* in, uint32_t n, uint16_t* table, uint32_t tsize,
                                      uint8_t* out, uint64_t op, uint32_t lane) {
  const uint32_t mask = tsize - 1;
  uint32_t ip = 0, next_emit = 0;
  if (n >= 15) {
    const uint32_t limit = n - 15;
    for (;;) {
      next_emit = ip++;
      uint32_t skip = 32, cand;
      for (;;) {
        const uint32_t data = uni(load32<kLds>(in, ip));
        const uint32_t h = hash_bytes(data, mask);
        const uint32_t step = skip >> 5;
        skip += step;
        const uint32_t next_ip = ip + step;
        if (next_ip > limit) {
          ip = next_emit;
          goto remainder;
        }
        cand = uni(table[h]);
        table[h] = (uint16_t)ip;
        if (uni(load32<kLds>(in, cand)) == data) break;
        ip = next_ip;
      }
      op = emit_literal(out, op, in + next_emit, ip - next_emit, lane);
      for (;;) {
        const uint32_t base = ip;
        const uint32_t matched = 4 + uni(match_len(in, cand + 4, ip + 4, n, lane));
        ip += matched;
        op = emit_copy(out, op, base - cand, matched, lane);
        next_emit = ip;
        if (ip >= limit) goto remainder;
        table[hash_bytes(uni(load32<kLds>(in, ip - 1)), mask)] = (uint16_t)(ip - 1);
        const uint32_t data = uni(load32<kLds>(in, ip));
        const uint32_t h = hash_bytes(data, mask);
        cand = uni(table[h]);
        table[h] = (uint16_t)ip;
        if (uni(load32<kLds>(in, cand)) != data) break;
      }
    }
  }
remainder:
  if (next_emit < n) op = emit_literal(out, op, in + next_emit, n - next_emit, lane);
  return op;
}

__global__ __launch_bounds__(kSnapThreads) void snappy_compress_kernel(SnapEncArgs a) {
  const uint32_t lane = threadIdx.x;
  uint16_t* const gtable = a.scratch + (uint64_t)blockIdx.x * kSnapMaxTable;
  for (uint64_t b = blockIdx.x; b < a.n; b += gridDim.x) {
    const uint64_t s = a.offsets[b];
    const uint64_t len = a.offsets[b + 1] - s;
    if (len >= 0xffffffffull) {
      if (lane == 0) a.out_len[b] = ~0ull;
      continue;
    }
    const uint32_t n = (uint32_t)len;
    uint8_t* const out = a.out + a.out_offsets[b];
    // varint32 preamble
    uint32_t pre = 1;
    while (pre < 5 && (n >> (7 * pre)) != 0) pre++;
    if (lane < pre) out[lane] = (uint8_t)(((n >> (7 * lane)) & 127u) | (lane + 1 < pre ? 128u : 0u));
    uint64_t op = pre;
    for (uint32_t pos = 0; pos < n; pos += kSnapFragment) {
      const uint32_t fn = n - pos < kSnapFragment ? n - pos : kSnapFragment;
      const uint32_t tsize = table_size_for(fn);
      const uint8_t* g = a.base + s + pos;
      if (2 * tsize + fn <= kSnapEncLds) {
        uint16_t* table = reinterpret_cast<uint16_t*>(smem);
        uint8_t* lin = smem + 2 * tsize;
        for (uint32_t j = lane; j < tsize / 2; j += 64) reinterpret_cast<uint32_t*>(smem)[j] = 0;
        for (uint32_t j = lane; j < fn; j += 64) lin[j] = g[j];
        wave_phase();
        op = compress_fragment<true>(lin, fn, table, tsize, out, op, lane);
        wave_phase();
      } else {
        for (uint32_t j = lane; j < tsize; j += 64) gtable[j] = 0;
        wave_phase();
        op = compress_fragment<false>(g, fn, gtable, tsize, out, op, lane);
        wave_phase();
      }
    }
    if (lane == 0) a.out_len[b] = op;
  }
}

}  // namespace

// ---- host-callable launchers (C++ linkage, used by snappy_engine.cc) ----
hipError_t launch_snappy_length(const SnapLenArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(snappy_length_kernel, dim3(grid), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_uncompress(const SnapDecArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(snappy_uncompress_kernel, dim3(grid), dim3(kSnapThreads), kSnapDecLds, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_compress(const SnapEncArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(snappy_compress_kernel, dim3(grid), dim3(kSnapThreads), kSnapEncLds, stream, a);
  return hipGetLastError();
}

}  // namespace lsbm
