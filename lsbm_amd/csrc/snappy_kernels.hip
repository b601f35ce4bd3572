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

typedef const __attribute__((address_space(1))) uint32_t* gcu32;  // global loads, not flat

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

// Compiler-only ordering for one wave's own LDS accesses (which the LDS
// executes in issue order): emits no wait.
__device__ __forceinline__ void wave_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// dst[0, n) = g[0, n) for a 4-aligned LDS dst and any global g: aligned
// dword loads (none past the dword holding g[n-1]), funnel-shifted into place,
// 4 per lane in flight.  The last dword's bytes past n are unspecified.
__device__ __forceinline__ void stage_to_lds(uint8_t* dst, const uint8_t* g, uint32_t n, uint32_t lane) {
  const uintptr_t ga = reinterpret_cast<uintptr_t>(g);
  const uint32_t sh = (uint32_t)(ga & 3u);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(ga - sh);
  const uint32_t nsrc = (sh + n + 3) >> 2;
  const uint32_t ndst = (n + 3) >> 2;
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (uint32_t k0 = 0; k0 < ndst; k0 += 256) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t k = k0 + u * 64 + lane;
      lo[u] = k < nsrc ? src[k] : 0u;
      hi[u] = k + 1 < nsrc ? src[k + 1] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t k = k0 + u * 64 + lane;
      if (k < ndst) d[k] = __builtin_amdgcn_alignbyte(hi[u], lo[u], sh);
    }
  }
}

// g[0, n) = src[0, n) from a 16-aligned LDS src: byte stores up to g's next
// 16-byte boundary, then 16-byte stores (five aligned LDS dwords per lane,
// funnel-shifted), then the < 16-byte tail.  Byte-wide global stores of a
// whole block cost a third of the decoder's time.
__device__ __forceinline__ void unstage_from_lds(uint8_t* g, const uint8_t* src, uint32_t n, uint32_t lane) {
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 15u);
  const uint32_t head = min(n, (16u - mis) & 15u);
  if (lane < head) g[lane] = src[lane];
  const uint32_t nq = (n - head) >> 4;
  const uint32_t sh = head & 3u;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(src + (head & ~3u));
  uint4* gd = reinterpret_cast<uint4*>(g + head);
  for (uint32_t q = lane; q < nq; q += 64) {
    const uint32_t* p = w + 4 * q;
    const uint32_t x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
    const uint32_t x4 = sh ? p[4] : 0u;  // holds needed bytes only when shifted
    gd[q] = make_uint4(__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                       __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
  }
  const uint32_t t = head + 16 * nq + lane;
  if (t < n) g[t] = src[t];
}

extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

// Phase timing of the encoder (diagnostic build only, -DLSBM_SNAP_STAMPS;
// tools/snappy_stamps.py): s_memtime deltas per phase, summed per wave.
#ifdef LSBM_SNAP_STAMPS
__device__ unsigned long long g_snap_stamps[16];  // 0-7 encoder phases, 9 encoder waves, 10-13 decoder, 15 decoder waves
struct Stamps {
  uint64_t t, acc[8];
};
#define SNAP_STAMP(k)                                    \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
    sa.acc[k] += t_ - sa.t;                              \
    sa.t = t_;                                           \
  } while (0)
#define SNAP_STAMPS_PARAM , Stamps& sa
#define SNAP_STAMPS_ARG , sa
#else
#define SNAP_STAMP(k) \
  do {                \
  } while (0)
#define SNAP_STAMPS_PARAM
#define SNAP_STAMPS_ARG
#endif

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

// load8 split in two, so that the two LDS dwords can be requested early and
// combined only where the value is needed (the shift would otherwise wait for
// the load right after issuing it).
struct Raw8 {
  uint64_t v;
  uint32_t sh;
};

template <bool kLds>
__device__ __forceinline__ Raw8 issue8(const uint8_t* p, uint32_t i, uint32_t n) {
  if (kLds) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (i & ~3u));
    return Raw8{(uint64_t)w[0] | ((uint64_t)w[1] << 32), 8 * (i & 3u)};
  } else {
    return Raw8{load8<false>(p, i, n), 0};
  }
}

__device__ __forceinline__ uint64_t finish8(Raw8 r) { return r.v >> r.sh; }

// 4 bytes at p[i] (the encoder's callers only ask for bytes inside the
// fragment).  Global memory: one unaligned dword load (gfx950 global loads
// take any byte alignment).
template <bool kLds>
__device__ __forceinline__ uint32_t load32(const uint8_t* p, uint32_t i) {
  if (kLds) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (i & ~3u));
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return (uint32_t)(v >> (8 * (i & 3u)));
  } else {
    typedef const __attribute__((address_space(1), aligned(1))) uint32_t* gu32u;
    return *reinterpret_cast<gu32u>(reinterpret_cast<uint64_t>(p) + i);
  }
}

// lane % d for lane < 64 and 1 <= d < 64 (an overlapping copy's source
// index): float reciprocal and one correction each way, not the integer
// division sequence.
__device__ __forceinline__ uint32_t lane_mod(uint32_t lane, uint32_t d) {
  const uint32_t q = (uint32_t)((float)lane * __builtin_amdgcn_rcpf((float)d));
  int32_t r = (int32_t)lane - (int32_t)(q * d);
  r = r < 0 ? r + (int32_t)d : (r >= (int32_t)d ? r - (int32_t)d : r);
  return (uint32_t)r;
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

// parse_preamble over the block's first bytes loaded at once: the two aligned
// dwords from the one holding p[0] (never a dword past the one holding
// p[n - 1]), so the varint costs one memory round trip, not one per byte.
__device__ __forceinline__ uint32_t parse_preamble_wide(const uint8_t* p, uint64_t n, uint32_t* ulen) {
  if (n == 0) return 0;
  const uint64_t g = reinterpret_cast<uint64_t>(p);
  const uint64_t a0 = g & ~3ull, last = (g + n - 1) & ~3ull;
  const uint32_t lo = *reinterpret_cast<gcu32>(a0);
  const uint32_t hi = *reinterpret_cast<gcu32>(a0 + 4 <= last ? a0 + 4 : a0);
  const uint64_t w = (((uint64_t)hi << 32) | lo) >> (8 * (uint32_t)(g & 3u));  // >= 5 valid bytes
  uint32_t v = 0;
  for (uint32_t i = 0; i < 5; i++) {
    if (i >= n) return 0;
    const uint32_t b = (uint32_t)(w >> (8 * i)) & 0xffu;
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
  // The input is read-only, so the next tag's word is requested before the
  // current tag's bytes move: the two LDS round trips overlap, and a tag costs
  // one wait instead of three.
  uint64_t w = ip < cl ? uni64(load8<kLds>(in, ip, cl)) : 0;
  while (ip < cl) {
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
      const uint32_t nip = ip + hdr + (uint32_t)len;
      const Raw8 wn = nip < cl ? issue8<kLds>(in, nip, cl) : Raw8{0, 0};
      for (uint32_t j = lane; j < (uint32_t)len; j += 64) dst[j] = src[j];
      ip = nip;
      op += (uint32_t)len;
      w = uni64(finish8(wn));
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
      const uint32_t nip = ip + hdr;
      const Raw8 wn = nip < cl ? issue8<kLds>(in, nip, cl) : Raw8{0, 0};
      // byte j of the copy is out[op - off + j mod off]: an overlapping copy
      // (off < len) repeats its first off bytes, all written before it.
      if (lane < len) {
        const uint32_t k = off >= len ? lane : lane_mod(lane, off);
        out[op + lane] = out[op - off + k];
      }
      ip = nip;
      op += len;
      w = uni64(finish8(wn));
    }
    // LDS variant: one wave's LDS accesses execute in issue order, so a copy
    // reads the bytes earlier tags wrote without waiting for the writes; the
    // wavefront-scope fence only keeps the compiler from reordering them.
    if (kLds) wave_order();
  }
  return op == ulen;
}

// The tag walk lane-parallel, 64 input bytes per step.  The windows are
// fixed: [ip, ip + 64), ip = 0, 64, 128, ... (a tag or a literal's data may
// straddle two of them).
//  1. Every lane parses the tag that WOULD start at its byte (branch-free:
//     kind, header size, length, offset).
//  2. A scalar walk over the real tags of the window (one readlane of each
//     tag's size and length) marks them in a 64-bit mask and hands each its
//     output offset (v_writelane): one scalar add per tag (an inline-asm
//     loop of 7 instructions; blocks of 16 KiB and more: the C loop).
//  3. Every real tag is checked at once against the conditions RawUncompress
//     tests (header or literal past the stream, offset 0 or before the output,
//     output past ulen).  The decode fails iff one of them fails: the tags up
//     to the first failing one are exactly the ones the serial walk visits,
//     and past it the result is "fail" whatever the rest holds.  Nothing is
//     written for a window with a failing tag, so a corrupt stream never
//     writes outside the output window.
//  4. Literal bytes: lane l owns input byte ip + l (the low byte of its parse
//     word); it belongs to the data of the last real tag at or before l, or,
//     below the window's first tag, to a literal that began in an earlier
//     window.  One byte store per lane, for every literal of the window.
//  5. Copies, in stream order, each spread over the lanes (one LDS round trip
//     each).  A copy reads only output before its own, written by earlier
//     copies or by literals (step 4, issued before).  (Pairing two copies per
//     round trip when the second reads nothing the first writes measured 6%
//     slower: profiles/r02/snappy/ab_lanes.log.)
// The compressed bytes are read from global memory (kGlobalIn: two aligned
// dwords per lane per window, requested one window ahead, through a buffer
// descriptor bounded to the dwords holding the stream), so the wave's LDS slice holds only the output
// window; or from an LDS copy (A/B builds).  Same accept / reject decisions as
// decode() (tests/test_snappy.py; tools/snappy_lanes_model.py restates the
// walk and checks it against the oracle).
template <bool kGlobalIn, bool kBig = false>
__device__ bool decode_lanes(const uint8_t* in, uint32_t cl, uint8_t* out, uint32_t ulen, uint32_t lane) {
  // > any valid length here: ulen < the slice (16 KiB; kBig: 80 KiB, where a
  // tag's size and output length no longer pack into one 32-bit word)
  constexpr uint32_t kLenCap = kBig ? 0x20000u : 0x4000u;
  uint32_t op = 0;    // output offset of the next tag
  uint32_t next = 0;  // input position of the next tag
  // a literal's data [lit_lo, lit_hi) that runs into later windows; out[lit_out] <- in[lit_lo]
  uint32_t lit_lo = 0, lit_hi = 0, lit_out = 0;
  // global input: a buffer descriptor over the dwords holding in[0, cl), so a
  // load past them returns zero without touching memory (no address clamps)
  const uint64_t gin = reinterpret_cast<uint64_t>(in);
  const uint32_t sh0 = (uint32_t)gin & 3u;
  __amdgpu_buffer_rsrc_t rsrc;
  if constexpr (kGlobalIn)
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in - sh0), (short)0,
                                             (int)((sh0 + cl + 3) & ~3u), 0x00020000);
  auto issue = [&](uint32_t i, uint32_t& lo, uint32_t& hi) {  // (global input only)
    const uint32_t a0 = (sh0 + i) & ~3u;
    lo = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, a0, 0, 0);
    hi = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, a0 + 4, 0, 0);
  };
  uint32_t lo = 0, hi = 0;
  if (kGlobalIn && cl) issue(lane, lo, hi);
  const uint64_t upto = ~0ull >> (63u - lane);  // lanes 0 .. lane
  for (uint32_t ip = 0; ip < cl; ip += 64) {
    uint64_t w;
    if constexpr (kGlobalIn) {
      uint32_t nlo, nhi;
      issue(ip + 64 + lane, nlo, nhi);  // the next window's words
      w = (((uint64_t)hi << 32) | lo) >> (8 * ((sh0 + ip + lane) & 3u));
      lo = nlo;
      hi = nhi;
    } else {
      w = load8<true>(in, ip + lane, cl);
    }
    // 1. the tag at this lane's byte, as selects (no per-kind branches)
    const uint32_t c = (uint32_t)w & 0xffu;
    const uint32_t x = (uint32_t)(w >> 8);  // the 4 bytes after the tag byte
    const uint32_t kind = c & 3u;
    const uint32_t len0 = (c >> 2) + 1;
    const uint32_t nb = len0 > 60 ? len0 - 60 : 0u;  // a literal's extra length bytes
    // the little-endian field after the tag byte: nb bytes (literal), 1 / 2 / 4 (copies)
    const uint32_t fb = kind == 0 ? nb : (kind == 3 ? 4u : kind);
    const uint32_t xm = fb == 4 ? x : x & ((1u << (8 * fb)) - 1u);
    const uint32_t len_lit = nb ? (xm == 0xffffffffu ? xm : xm + 1) : len0;  // (saturated: fails anyway)
    const uint32_t hdr = 1 + fb;
    const uint32_t len = kind == 0 ? len_lit : (kind == 1 ? 4 + ((c >> 2) & 7u) : len0);
    const uint32_t off = kind == 1 ? ((c >> 5) << 8) | xm : xm;
    const uint32_t lenc = len < kLenCap ? len : kLenCap;
    const uint32_t size = hdr + (kind == 0 ? lenc : 0u);
    const uint32_t ws = kBig ? size : size | (lenc << 16);  // size | output length
    // 2. the real tags of this window and their output offsets (from op)
#ifndef LSBM_SNAP_SCALAR_MASK  // (A/B builds: the mask built by two scalar ops per tag, 4% slower)
    // the real tags are the lanes the walk writes: opt starts at ~0 (never a
    // real tag's offset) and the mask is one ballot after the walk, not two
    // scalar ops per tag
    uint32_t opt = ~0u, opa = 0;
#else
    uint64_t real = 0;
    uint32_t opt = 0, opa = 0;
#endif
    uint32_t s = next - ip;
    const uint32_t lim = cl - ip;
#if !defined(LSBM_SNAP_SCALAR_MASK) && !defined(LSBM_SNAP_C_WALK)
    if constexpr (!kBig) {
      // the walk as 7 instructions per tag: one scalar accumulator
      // acc = opa << 16 | s (s < 2^16; opa < 2^16 up to the first tag whose
      // output passes ulen < 16 KiB, which fails its check) advanced by one
      // add of the packed size | output length; the lane select is acc's low
      // half in M0; each real lane receives acc (opa in its high half)
      // (readfirstlane: both are wave-uniform; it tells the compiler so)
      const uint32_t lim64 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lim < 64u ? lim : 64u));
      uint32_t acc = (uint32_t)__builtin_amdgcn_readfirstlane((int)s), v;
      asm volatile(
          "s_and_b32 m0, %[acc], 0xffff\n\t"
          "s_cmp_lt_u32 m0, %[lim]\n\t"
          "s_cbranch_scc0 2f\n"
          "1:\n\t"
          "v_writelane_b32 %[opt], %[acc], m0\n\t"
          "v_readlane_b32 %[v], %[ws], m0\n\t"
          "s_add_u32 %[acc], %[acc], %[v]\n\t"
          "s_and_b32 m0, %[acc], 0xffff\n\t"
          "s_cmp_lt_u32 m0, %[lim]\n\t"
          "s_cbranch_scc1 1b\n"
          "2:"
          : [acc] "+s"(acc), [opt] "+v"(opt), [v] "=&s"(v)
          : [ws] "v"(ws), [lim] "s"(lim64)
          : "m0", "scc");
      (void)v;
      s = acc & 0xffffu;
      opa = acc >> 16;
      opt = opt == ~0u ? opt : opt >> 16;
    } else
#endif
    while (s < 64u && s < lim) {
#ifdef LSBM_SNAP_SCALAR_MASK
      real |= 1ull << s;
#endif
      // opt[s] = opa: v_writelane (one VALU instead of a compare and a select;
      // lane select in M0, which no other instruction of these kernels uses --
      // gfx9's constant bus takes one SGPR besides M0)
      asm("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(opt) : "s"(opa), "s"(s) : "m0");
      const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)ws, (int)s);
      if constexpr (kBig) {
        opa += (uint32_t)__builtin_amdgcn_readlane((int)lenc, (int)s);
        s += v;
      } else {
        opa += v >> 16;
        s += v & 0xffffu;
      }
    }
#ifndef LSBM_SNAP_SCALAR_MASK
    const uint64_t real = __ballot(opt != ~0u);
#endif
    const uint32_t o = op + opt;
    if (real) {
      // 3. every real tag's checks (a literal's extra length bytes past the
      // stream are hdr > rem, like a copy's offset bytes)
      const uint32_t rem = cl - (ip + lane);  // >= 1 on a real tag's lane
      // the kind's own test as one compare ka >= kb: a literal's data past the
      // stream (len > rem - hdr; rem - hdr + 1 wraps only when hdr > rem,
      // which fails anyway), a copy's offset 0 or before the output
      // (off - 1 >= o).  Bitwise, not short-circuit: no divergent branches.
      const uint32_t ka = kind == 0 ? len : off - 1u;
      const uint32_t kb = kind == 0 ? rem - hdr + 1u : o;
      const bool bad = (hdr > rem) | (len > ulen - o) | (ka >= kb);
      if (__ballot(bad) & real) return false;
    }
    // 4. literal bytes: the tag owning this lane's byte (the last real tag at
    // or before it) and its data range, or the literal carried in
    const uint32_t pack = kind | (hdr << 2) | ((len < 127u ? len : 127u) << 5) | (opt << 12);
    const uint64_t below = real & upto;
    const uint32_t own = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
    const uint32_t po = (uint32_t)__shfl((int)pack, (int)own);
    // (selects, not a branch: below is 0 only on lanes before the window's first tag)
    const uint32_t d0 = ip + own + ((po >> 2) & 7u);
    const uint32_t d1 = (po & 3u) == 0 ? d0 + ((po >> 5) & 127u) : d0;  // (a copy owns no data)
    const bool hb = below != 0;
    const uint32_t dlo = hb ? d0 : lit_lo, dhi = hb ? d1 : lit_hi, dout = hb ? op + (po >> 12) : lit_out;
    const uint32_t pos = ip + lane;
    if (pos >= dlo && pos < dhi) out[dout + (pos - dlo)] = (uint8_t)c;
    if (real) {  // the last tag's literal data may run into the next windows
      const uint32_t t = 63u - (uint32_t)__builtin_clzll(real);
      const uint32_t tp = (uint32_t)__builtin_amdgcn_readlane((int)pack, (int)t);
      const uint32_t tl = (uint32_t)__builtin_amdgcn_readlane((int)(kBig ? lenc : ws >> 16), (int)t);
      lit_lo = ip + t + ((tp >> 2) & 7u);
      lit_hi = (tp & 3u) == 0 ? lit_lo + tl : lit_lo;
      lit_out = op + (tp >> 12);
    }
    // 5. the copies, in order: output [dst, dst + len) from [dst - off, ...)
    constexpr uint32_t kOB = kBig ? 17u : 16u;  // bits of a valid copy's output offset (o < ulen)
    // packed per copy: output offset | (len - 1) << kOB | overlapping (off < len) << 23
    const uint32_t cpa = o | ((len - 1) << kOB) | (off < len ? 1u << 23 : 0u);  // (len <= 64)
    const uint32_t cps = o - off;
    uint64_t cm = real & __ballot(kind != 0);
    while (cm) {
      wave_order();
      const uint32_t t = (uint32_t)__builtin_ctzll(cm);
      cm ^= 1ull << t;
      const uint32_t ta = (uint32_t)__builtin_amdgcn_readlane((int)cpa, (int)t);
      const uint32_t src = (uint32_t)__builtin_amdgcn_readlane((int)cps, (int)t);
      const uint32_t dst = ta & ((1u << kOB) - 1u), tlen = ((ta >> kOB) & 63u) + 1;
      // byte j of the copy is out[src + j mod off]: an overlapping copy
      // (off < len) repeats its first off bytes, all written before it
      if (lane < tlen) {
        const uint32_t k = (ta >> 23) & 1u ? lane_mod(lane, dst - src) : lane;
        out[dst + lane] = out[src + k];
      }
    }
    wave_order();
    op += opa;
    next = ip + s;
  }
  return op == ulen;
}

// Decodes block b into the wave's LDS slice of kSlice bytes when its output
// fits (the compressed bytes are read from global memory; A/B builds with
// LSBM_SNAP_STAGED_INPUT stage them in the slice too), else
// (kGlobalFallback) against global memory.  Returns 2 when the block neither
// fits nor may fall back.
template <uint32_t kSlice, bool kGlobalFallback, uint32_t kDefer = 2>
__device__ __forceinline__ uint32_t uncompress_block(const SnapDecArgs& a, uint64_t b, uint32_t lane
                                                     SNAP_STAMPS_PARAM) {
  const uint64_t s = a.offsets[b], e = a.offsets[b + 1];
  const uint64_t os = a.out_offsets[b], cap = a.out_offsets[b + 1] - os;
  const uint64_t clen = e - s;
  uint32_t ulen = 0;
  const uint32_t pre = uni(parse_preamble_wide(a.base + s, clen, &ulen));
  ulen = uni(ulen);
  if (pre == 0 || (uint64_t)ulen > cap) return 0;
  const uint64_t cl64 = clen - pre;
  if (cl64 >= 0xffffffffull) return 0;  // a >= 4 GiB compressed block (snappy's lengths are 32-bit)
  const uint8_t* g = a.base + s + pre;
  const uint32_t cl = (uint32_t)cl64;
  bool ok;
#ifdef LSBM_SNAP_STAGED_INPUT  // A/B builds only: the compressed bytes staged in the slice too
  const uint64_t need = cl64 + 8 + 15 + (uint64_t)ulen;
#else
  const uint64_t need = (uint64_t)ulen + 16;  // (unstage_from_lds reads up to 16 B past ulen)
#endif
  if (need <= kSlice) {
    SNAP_STAMP(0);  // offsets + preamble
#ifdef LSBM_SNAP_STAGED_INPUT
    uint8_t* const lds_in = smem;
    stage_to_lds(lds_in, g, cl, lane);
    wave_order();
    if (lane < 8) lds_in[cl + lane] = 0;  // zero pad behind the stream (load8 reads <= cl+6)
    uint8_t* win = smem + (uint32_t)((cl64 + 8 + 15) & ~15ull);
    wave_phase();
    ok = decode_lanes<false>(lds_in, cl, win, ulen, lane);
#else
    uint8_t* win = smem;
    ok = decode_lanes<true, (kSlice > 16384)>(g, cl, win, ulen, lane);  // (kBig: ulen >= 16 KiB possible)
#endif
    SNAP_STAMP(2);
#ifndef LSBM_SNAP_DIAG_NO_OUT  // diagnostic build only (tools/snappy_diag.py): skips the output, wrong results
    if (ok) unstage_from_lds(a.out + os, win, ulen, lane);
#endif
    SNAP_STAMP(3);
    wave_phase();
  } else if (!kGlobalFallback) {
    return kDefer;
  } else {
    ok = decode<false>(g, cl, a.out + os, ulen, lane);
  }
  return ok ? 1 : 0;
}

__device__ __forceinline__ void record(const SnapDecArgs& a, uint64_t b, uint32_t r, uint32_t lane) {
  if (lane == 0) {
    a.ok[b] = (uint8_t)r;
    if (r == 0 && a.n_bad) atomicAdd(a.n_bad, 1u);
  }
}

// Pass 1: every block that fits a small slice (a db_bench data block and its
// compressed form need < 7 KiB), at kSnapDecWgsPerCu waves per CU; the rest
// are marked ok = 2 for pass 2.
__global__ __launch_bounds__(kSnapThreads) void snappy_uncompress_kernel(SnapDecArgs a) {
  const uint32_t lane = threadIdx.x;
#ifdef LSBM_SNAP_STAMPS
  Stamps sa = {};
  sa.t = __builtin_amdgcn_s_memtime();
#endif
  for (uint64_t b = blockIdx.x; b < a.n; b += gridDim.x)
    record(a, b, uncompress_block<kSnapDecLds, false>(a, b, lane SNAP_STAMPS_ARG), lane);
#ifdef LSBM_SNAP_STAMPS
  if (lane == 0) {
    for (int k = 0; k < 4; k++) atomicAdd(&g_snap_stamps[10 + k], (unsigned long long)sa.acc[k]);
    atomicAdd(&g_snap_stamps[15], 1ull);
  }
#endif
}

// Passes 2-5: the blocks the pass before deferred (ok = kPending), found 64
// at a time by ballot, in 9 / 17 / 33 / 80 KiB output windows (17 / 9 / 4 / 2
// waves per CU: blocks of 8, 16, 32 and 64 KiB block sizes, which run a little
// over), each deferring what does not fit (ok = kPending + 1) and the last
// decoding the rest serially against global memory (decode<false>).  (With a
// 16 KiB pass only, blocks of 16-64 KiB went straight to the serial path:
// 8.6 GB/s on 62 KB db_bench-like blocks, profiles/r02/snappy/merge_blocks.log.)
template <uint32_t kSlice, uint32_t kPending, bool kFallback>
__global__ __launch_bounds__(kSnapThreads) void snappy_uncompress_deferred_kernel(SnapDecArgs a) {
  const uint32_t lane = threadIdx.x;
  // 16 blocks per scan, so that a batch of larger blocks (all deferred) still
  // gives every wave slot of the pass work: 64 per scan left 8 of 17 waves
  // per CU busy on 8 KB blocks
  constexpr uint32_t kScan = kSnapDecScan;
  for (uint64_t c = (uint64_t)blockIdx.x * kScan; c < a.n; c += (uint64_t)gridDim.x * kScan) {
    const uint64_t i = c + lane;
    uint64_t pend = __ballot(lane < kScan && i < a.n && a.ok[i] == kPending);
    while (pend) {
      const uint64_t b = c + (uint64_t)__builtin_ctzll(pend);
      pend &= pend - 1;
#ifdef LSBM_SNAP_STAMPS
      Stamps sa = {};
#endif
      record(a, b, uncompress_block<kSlice, kFallback, kPending + 1>(a, b, lane SNAP_STAMPS_ARG), lane);
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
// Lane k's probe of a match search whose first probe is at p with skip sc:
// probe k+1 = probe k + (skip_k >> 5), skip_{k+1} = skip_k + (skip_k >> 5).
__device__ __forceinline__ void probe_positions(uint32_t p, uint32_t sc, uint32_t lane, uint32_t* pk,
                                                uint32_t* sk) {
  for (uint32_t j = 0; j < 64; j++) {
    if (lane == j) {
      *pk = p;
      *sk = sc;
    }
    const uint32_t st = sc >> 5;
    p += st;
    sc += st;
  }
}

template <bool kLds>
__device__ uint64_t compress_fragment(const uint8_t* in, uint32_t n, uint16_t* table, uint32_t tsize,
                                      uint8_t* out, uint64_t op, uint32_t lane, uint32_t off32,
                                      uint32_t sk32, uint32_t off64, uint32_t sk64,
                                      uint32_t* buckets SNAP_STAMPS_PARAM) {
  const uint32_t mask = tsize - 1;
  uint32_t ip = 0, next_emit = 0;
  if (n >= 15) {
    const uint32_t limit = n - 15;
    for (;;) {
      next_emit = ip++;
      SNAP_STAMP(4);
      uint32_t cand;
      // The search's probe positions depend only on where it starts (skip
      // restarts at 32), so the wave makes 64 probes at once, lane k taking
      // probe k.  What the serial walk's table read would return for probe k
      // is the position of the latest earlier lane with the same hash, if any,
      // else the table's value; the first lane whose candidate matches is the
      // serial walk's match, and lanes up to it update the table (the last
      // writer of each hash only).
      const uint32_t start = ip;
      uint32_t k0 = 0;
      uint32_t pk = ip + off32, sk = sk32;
      for (;;) {
        const uint32_t step = sk >> 5;
        const bool valid = lane < kSnapProbes && pk + step <= limit;
        const uint32_t data = load32<kLds>(in, valid ? pk : 0);
        const uint32_t h = hash_bytes(data, mask);
        const uint32_t old = table[h];
        // Lanes sharing a hash share one of kSnapEncBuckets LDS counters; only
        // lanes whose counter reached 2 can have a same-hash peer.
        // (8-bit counters, four to a dword: a batch counts at most 64)
        const uint32_t bk = h & (kSnapEncBuckets - 1);
        uint32_t* const cnt = buckets + (bk >> 2);
        const uint32_t bsh = 8 * (bk & 3u);
        if (valid) atomicAdd(cnt, 1u << bsh);
        const uint32_t nb = valid ? (*cnt >> bsh) & 0xffu : 0u;
        if (valid) *cnt = 0u;
        const uint64_t flagged = __ballot(nb >= 2);
        SNAP_STAMP(6);
        // a lane with no peer matches iff the table's candidate does
        const bool m0 = valid && load32<kLds>(in, valid ? old : 0) == data;
        const uint64_t vm = __ballot(valid);
        const uint64_t mm0 = __ballot(m0) & ~flagged;
        const uint32_t lnf = mm0 ? (uint32_t)__builtin_ctzll(mm0) : 64u;
        // Flagged lanes in ascending order.  When the walk reaches lane j, j's
        // latest same-hash predecessor is final, and with it j's candidate;
        // a predecessor holds the same hash, so j matches iff their 4 bytes
        // agree (data in registers, no load).  The walk stops at the first
        // flagged match or past the first unflagged one: later lanes do not
        // matter.  st: bit 0 = has a predecessor, bit 1 = its bytes agree.
        uint32_t pred = 64, succ = 64, st = 0;
        uint32_t last = lnf;
        for (uint64_t f = flagged; f;) {
          const uint32_t j = (uint32_t)__builtin_ctzll(f);
          f &= f - 1;
          if (j > lnf) break;
          const uint32_t hj = __builtin_amdgcn_readlane(h, j);
          const uint32_t dj = __builtin_amdgcn_readlane(data, j);
          const uint32_t sj = __builtin_amdgcn_readlane(st, j);
          const bool mj = (sj & 1u) ? (sj & 2u) != 0 : __builtin_amdgcn_readlane((uint32_t)m0, j) != 0;
          // branch-free updates (selects, no divergent branches)
          const bool eq = hj == h;
          const bool after = eq && lane > j;
          pred = after ? j : pred;
          st = after ? (dj == data ? 3u : 1u) : st;
          succ = (eq && lane < j && succ == 64) ? j : succ;
          if (mj) {
            last = j;
            break;
          }
        }
        SNAP_STAMP(7);
        constexpr uint64_t kAll = kSnapProbes == 64 ? ~0ull : (1ull << kSnapProbes) - 1;
        if (last == 64 && vm != kAll) {  // the search reached the limit
          ip = next_emit;
          goto remainder;
        }
        const uint64_t mm = last < 64 ? 1ull : 0ull;
        if (last == 64) last = kSnapProbes - 1;
        if (lane <= last && succ > last) table[h] = (uint16_t)pk;
        // later reads of these entries come from other lanes: in LDS the
        // wave's accesses run in order; in global memory wait for the stores
        if (kLds) wave_order();
        else wave_phase();
        if (mm) {
          ip = __builtin_amdgcn_readlane(pk, last);
          const uint32_t pl = __builtin_amdgcn_readlane(pred, last);
          cand = pl < 64 ? __builtin_amdgcn_readlane(pk, pl) : __builtin_amdgcn_readlane(old, last);
          break;
        }
        // next step: probes k0 + lane of the search, from the per-wave tables
        // of the first 128 (a search's probe offsets do not depend on where
        // it starts), else by the serial recurrence
        k0 += kSnapProbes;
        if (k0 + kSnapProbes <= 128) {
          const int src = (int)((k0 + lane) & 63u);
          const uint32_t oa = (uint32_t)__shfl((int)off32, src), ob = (uint32_t)__shfl((int)off64, src);
          const uint32_t sa = (uint32_t)__shfl((int)sk32, src), sb = (uint32_t)__shfl((int)sk64, src);
          const bool hi = k0 + lane >= 64;
          pk = start + (hi ? ob : oa);
          sk = hi ? sb : sa;
        } else {
          const uint32_t pl = __builtin_amdgcn_readlane(pk, kSnapProbes - 1);
          const uint32_t sl = __builtin_amdgcn_readlane(sk, kSnapProbes - 1);
          probe_positions(pl + (sl >> 5), sl + (sl >> 5), lane, &pk, &sk);
        }
      }
      SNAP_STAMP(1);
      op = emit_literal(out, op, in + next_emit, ip - next_emit, lane);
      SNAP_STAMP(2);
      for (;;) {
        const uint32_t base = ip;
        const uint32_t matched = 4 + uni(match_len(in, cand + 4, ip + 4, n, lane));
        ip += matched;
        op = emit_copy(out, op, base - cand, matched, lane);
        SNAP_STAMP(3);
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
  SNAP_STAMP(4);
  if (next_emit < n) op = emit_literal(out, op, in + next_emit, n - next_emit, lane);
  SNAP_STAMP(5);
  return op;
}

// Per-wave setup shared by both encoder passes: lane k's offsets and skips of
// probes k and 64 + k of a search from position 0 (skip 32), and the zeroed
// hash-bucket counters at `buckets`.
struct EncWave {
  uint32_t off32, sk32, off64, sk64;
  uint32_t* buckets;
};

__device__ __forceinline__ EncWave enc_wave(uint32_t* buckets, uint32_t lane) {
  EncWave w;
  probe_positions(0, 32, lane, &w.off32, &w.sk32);
  const uint32_t p63 = __builtin_amdgcn_readlane(w.off32, 63), s63 = __builtin_amdgcn_readlane(w.sk32, 63);
  probe_positions(p63 + (s63 >> 5), s63 + (s63 >> 5), lane, &w.off64, &w.sk64);
  w.buckets = buckets;
  for (uint32_t j = lane; j < kSnapEncBuckets / 4; j += 64) buckets[j] = 0;  // zero between searches
  wave_order();
  return w;
}

// varint32 preamble of block b; returns its size
__device__ __forceinline__ uint32_t write_preamble(uint8_t* out, uint32_t n, uint32_t lane) {
  uint32_t pre = 1;
  while (pre < 5 && (n >> (7 * pre)) != 0) pre++;
  if (lane < pre) out[lane] = (uint8_t)(((n >> (7 * lane)) & 127u) | (lane + 1 < pre ? 128u : 0u));
  return pre;
}

// Pass 1: every block that is one fragment fitting the wave's 22 KiB slice
// (fragment bytes and table in LDS, 7 waves per CU).  Larger blocks are
// marked kSnapDeferred for pass 2.
__global__ __launch_bounds__(kSnapThreads) void snappy_compress_kernel(SnapEncArgs a) {
  const uint32_t lane = threadIdx.x;
  const EncWave w = enc_wave(reinterpret_cast<uint32_t*>(smem + kSnapEncSlice), lane);
#ifdef LSBM_SNAP_STAMPS
  Stamps sa = {};
  sa.t = __builtin_amdgcn_s_memtime();
#endif
  for (uint64_t b = blockIdx.x; b < a.n; b += gridDim.x) {
    const uint64_t s = a.offsets[b];
    const uint64_t len = a.offsets[b + 1] - s;
    if (len >= 0xffffffffull) {
      if (lane == 0) a.out_len[b] = ~0ull;
      continue;
    }
    const uint32_t n = (uint32_t)len;
    const uint32_t tsize = table_size_for(n);
    if (n > kSnapFragment || 2 * tsize + n + 4 > kSnapEncSlice) {  // + the staged copy's last dword
      if (lane == 0) a.out_len[b] = kSnapDeferred;
      continue;
    }
    uint8_t* const out = a.out + a.out_offsets[b];
    const uint64_t op = write_preamble(out, n, lane);
    uint16_t* table = reinterpret_cast<uint16_t*>(smem);
    uint8_t* lin = smem + 2 * tsize;
    for (uint32_t j = lane; j < tsize / 8; j += 64) reinterpret_cast<uint4*>(smem)[j] = make_uint4(0, 0, 0, 0);
    stage_to_lds(lin, a.base + s, n, lane);
    wave_phase();
    SNAP_STAMP(0);  // staging, table zeroing, preamble
    const uint64_t end = compress_fragment<true>(lin, n, table, tsize, out, op, lane, w.off32, w.sk32, w.off64,
                                                 w.sk64, w.buckets SNAP_STAMPS_ARG);
    wave_phase();
    if (lane == 0) a.out_len[b] = end;
  }
#ifdef LSBM_SNAP_STAMPS
  if (lane == 0) {
    for (int k = 0; k < 8; k++) atomicAdd(&g_snap_stamps[k], (unsigned long long)sa.acc[k]);
    atomicAdd(&g_snap_stamps[9], 1ull);
  }
#endif
}

// Middle pass: deferred blocks of one fragment whose table and bytes fit a
// 48 KiB slice (up to ~16 KiB: a 2^14-entry table and the fragment in LDS,
// 3 waves per CU), the same code as pass 1; the rest stay deferred for the
// last pass.  (Without it every block past pass 1's 22 KiB slice went to the
// last pass, 2 waves per CU with the fragment read from global memory:
// profiles/r02/snappy/merge_blocks.log.)
__global__ __launch_bounds__(kSnapThreads) void snappy_compress_mid_kernel(SnapEncArgs a) {
  const uint32_t lane = threadIdx.x;
  const EncWave w = enc_wave(reinterpret_cast<uint32_t*>(smem + kSnapEncMidSlice), lane);
#ifdef LSBM_SNAP_STAMPS
  Stamps sa = {};
  sa.t = __builtin_amdgcn_s_memtime();
#endif
  for (uint64_t c = (uint64_t)blockIdx.x * kSnapDecScan; c < a.n; c += (uint64_t)gridDim.x * kSnapDecScan) {
    const uint64_t i = c + lane;
    uint64_t pend = __ballot(lane < kSnapDecScan && i < a.n && a.out_len[i] == kSnapDeferred);
    while (pend) {
      const uint64_t b = c + (uint64_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t s = a.offsets[b];
      const uint64_t len = a.offsets[b + 1] - s;
      if (len > kSnapFragment) continue;  // (pass 1 handled lengths >= 2^32)
      const uint32_t n = (uint32_t)len;
      const uint32_t tsize = table_size_for(n);
      if (2 * tsize + n + 4 > kSnapEncMidSlice) continue;  // + the staged copy's last dword
      uint8_t* const out = a.out + a.out_offsets[b];
      const uint64_t op = write_preamble(out, n, lane);
      uint16_t* table = reinterpret_cast<uint16_t*>(smem);
      uint8_t* lin = smem + 2 * tsize;
      for (uint32_t j = lane; j < tsize / 8; j += 64) reinterpret_cast<uint4*>(smem)[j] = make_uint4(0, 0, 0, 0);
      stage_to_lds(lin, a.base + s, n, lane);
      wave_phase();
      const uint64_t end = compress_fragment<true>(lin, n, table, tsize, out, op, lane, w.off32, w.sk32, w.off64,
                                                   w.sk64, w.buckets SNAP_STAMPS_ARG);
      wave_phase();
      if (lane == 0) a.out_len[b] = end;
    }
  }
}

// Pass 2: the deferred blocks, found 64 at a time by ballot, fragment by
// 64 KiB fragment: the hash table (up to 2^15 entries, 64 KiB) in LDS, the
// fragment bytes read from global memory.  No global scratch.
__global__ __launch_bounds__(kSnapThreads) void snappy_compress_large_kernel(SnapEncArgs a) {
  const uint32_t lane = threadIdx.x;
  const EncWave w = enc_wave(reinterpret_cast<uint32_t*>(smem + 2 * kSnapMaxTable), lane);
  uint16_t* const table = reinterpret_cast<uint16_t*>(smem);
#ifdef LSBM_SNAP_STAMPS
  Stamps sa = {};
  sa.t = __builtin_amdgcn_s_memtime();
#endif
  for (uint64_t c = (uint64_t)blockIdx.x * kSnapDecScan; c < a.n; c += (uint64_t)gridDim.x * kSnapDecScan) {
    const uint64_t i = c + lane;
    uint64_t pend = __ballot(lane < kSnapDecScan && i < a.n && a.out_len[i] == kSnapDeferred);
    while (pend) {
      const uint64_t b = c + (uint64_t)__builtin_ctzll(pend);
      pend &= pend - 1;
      const uint64_t s = a.offsets[b];
      const uint32_t n = (uint32_t)(a.offsets[b + 1] - s);
      uint8_t* const out = a.out + a.out_offsets[b];
      uint64_t op = write_preamble(out, n, lane);
      for (uint32_t pos = 0; pos < n; pos += kSnapFragment) {
        const uint32_t fn = n - pos < kSnapFragment ? n - pos : kSnapFragment;
        const uint32_t tsize = table_size_for(fn);
        for (uint32_t j = lane; j < tsize / 8; j += 64) reinterpret_cast<uint4*>(smem)[j] = make_uint4(0, 0, 0, 0);
        wave_phase();
        op = compress_fragment<false>(a.base + s + pos, fn, table, tsize, out, op, lane, w.off32, w.sk32, w.off64,
                                      w.sk64, w.buckets SNAP_STAMPS_ARG);
        wave_phase();
      }
      if (lane == 0) a.out_len[b] = op;
    }
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

// the deferred decode passes, in order (snappy_types.h kSnapDecTierLds)
template <int kTier>
hipError_t launch_deferred_tier(const SnapDecArgs& a, int grid, hipStream_t stream) {
  constexpr uint32_t lds = kSnapDecTierLds[kTier];
  constexpr bool last = kTier + 1 == kSnapDecTiers;
  auto* k = snappy_uncompress_deferred_kernel<lds, 2 + kTier, last>;
  if (lds > 65536) {  // above the default dynamic limit, within gfx950's 160 KiB per workgroup
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(kSnapThreads), lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_uncompress_deferred(const SnapDecArgs& a, int tier, int grid, hipStream_t stream) {
  static_assert(kSnapDecTiers == 4, "one case per tier");
  switch (tier) {
    case 0: return launch_deferred_tier<0>(a, grid, stream);
    case 1: return launch_deferred_tier<1>(a, grid, stream);
    case 2: return launch_deferred_tier<2>(a, grid, stream);
    default: return launch_deferred_tier<3>(a, grid, stream);
  }
}

hipError_t launch_snappy_compress(const SnapEncArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(snappy_compress_kernel, dim3(grid), dim3(kSnapThreads), kSnapEncLds, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_compress_mid(const SnapEncArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(snappy_compress_mid_kernel, dim3(grid), dim3(kSnapThreads), kSnapEncMidLds, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_compress_large(const SnapEncArgs& a, int grid, hipStream_t stream) {
  // 64.5 KiB of dynamic LDS: above the default dynamic limit, within gfx950's
  // 160 KiB per workgroup
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&snappy_compress_large_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSnapEncLargeLds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(snappy_compress_large_kernel, dim3(grid), dim3(kSnapThreads), kSnapEncLargeLds, stream, a);
  return hipGetLastError();
}

}  // namespace lsbm

#ifdef LSBM_SNAP_STAMPS
extern "C" __attribute__((visibility("default"))) int lsbm_snappy_debug_stamps(unsigned long long* out16,
                                                                                int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(lsbm::g_snap_stamps), 16 * sizeof(unsigned long long)) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lsbm::g_snap_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
