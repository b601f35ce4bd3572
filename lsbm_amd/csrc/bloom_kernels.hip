// bloom_kernels.hip -- gfx950 kernels of the batched bloom-filter engine
// (include/lsbm_bloom.h).
//
// bloom_build_kernel  CreateFilter (util/bloom.cc:37-63) for many filters:
//                     one wave per filter.  The wave's lanes hash one key
//                     each and set the key's k bits with ds_or_b32 in the
//                     wave's LDS slice; the finished bit array leaves LDS once,
//                     as dword stores (byte stores at the two unaligned ends,
//                     which may share a dword with a neighbouring filter).
//                     Filters wider than the slice are built window by window
//                     (every key re-hashed per window; rare: > 1,600 keys at
//                     20 bits/key).  No global atomics, no zero-fill pass.
// bloom_probe_kernel  KeyMayMatch (util/bloom.cc:65-89) for many lookups, one
//                     lane per lookup, optionally through FilterBlockReader's
//                     offset array (table/filter_block.cc:78-109).
//
// Both hash exactly as util/hash.cc:18-49, signed-char tail included, and
// take bitpos = h % bits as util/bloom.cc:58/84 do (32-bit h, size_t bits).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_types.h"

namespace lsbm {
namespace {

typedef const __attribute__((address_space(1))) uint32_t* gcu32;
typedef const __attribute__((address_space(1))) uint8_t* gcu8;
typedef __attribute__((address_space(1))) uint32_t* gu32;
typedef __attribute__((address_space(1))) uint8_t* gu8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gcu32x4;

constexpr uint32_t kHashM = 0xc6a4a793u;     // util/hash.cc:20
constexpr uint32_t kBloomSeed = 0xbc9f1d34u;  // util/bloom.cc:14

// A `char` of util/hash.cc:37-43, promoted to int and then to uint32_t.
__device__ __forceinline__ uint32_t sext8(uint32_t b) { return (uint32_t)(int32_t)(int8_t)(uint8_t)b; }

// util/hash.cc:18-49 over global bytes [s, s + n), any alignment.  Words are
// read aligned and funnel-shifted (v_alignbyte); only words that overlap the
// key are read, so a key ending at a page boundary never touches the next page.
__device__ uint32_t hash_key(uint64_t s, uint64_t n, uint32_t seed) {
  uint32_t h = seed ^ (uint32_t)(n * kHashM);
  if (n == 0) return h;
  const uint64_t w_last = (s + n - 1) & ~3ull;
  const uint32_t sh = (uint32_t)s & 3u;
  uint64_t q = s & ~3ull;
  uint32_t lo = *reinterpret_cast<gcu32>(q);
  for (uint64_t k = n >> 2; k; k--) {  // 4-byte steps (:26-32)
    q += 4;
    const uint32_t hi = *reinterpret_cast<gcu32>(q < w_last ? q : w_last);
    h += __builtin_amdgcn_alignbyte(hi, lo, sh);
    h *= kHashM;
    h ^= h >> 16;
    lo = hi;
  }
  const uint32_t r = (uint32_t)n & 3u;
  if (r) {  // the byte tail (:35-47)
    q += 4;
    const uint32_t hi = *reinterpret_cast<gcu32>(q < w_last ? q : w_last);
    const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, sh);
    if (r == 3) h += sext8(w >> 16) << 16;
    if (r >= 2) h += sext8(w >> 8) << 8;
    h += sext8(w);
    h *= kHashM;
    h ^= h >> 24;
  }
  return h;
}

// The same hash for latency-bound callers (the probe kernel): the words of up
// to 8 steps (32 key bytes) are all requested before the first is used, so a
// key costs one memory round trip per 32 bytes instead of one per 4 (a
// db_bench user key, 23 B, is one round trip).  More VALU than hash_key.
__device__ uint32_t hash_key_batched(uint64_t s, uint64_t n, uint32_t seed) {
  uint32_t h = seed ^ (uint32_t)(n * kHashM);
  if (n == 0) return h;
  const uint64_t w0 = s & ~3ull, w_last = (s + n - 1) & ~3ull;
  const uint32_t sh = (uint32_t)s & 3u;
  const uint64_t full = n >> 2;
  const uint32_t r = (uint32_t)n & 3u;
  const uint64_t steps = full + (r ? 1 : 0);
  for (uint64_t c = 0; c < steps; c += 8) {
    uint32_t w[9];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t q = w0 + 4 * (c + j);
      w[j] = *reinterpret_cast<gcu32>(q < w_last ? q : w_last);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = c + j;
      const uint32_t x = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
      if (t < full) {
        h += x;
        h *= kHashM;
        h ^= h >> 16;
      } else if (t == full && r) {
        if (r == 3) h += sext8(x >> 16) << 16;
        if (r >= 2) h += sext8(x >> 8) << 8;
        h += sext8(x);
        h *= kHashM;
        h ^= h >> 24;
      }
    }
  }
  return h;
}

// The same hash over a key staged in LDS: byte `rel` of the wave's staging
// area `stg` (words past the key may be read; they only feed bytes the tail
// step drops).  One address, immediate word offsets, no clamps.
__device__ __forceinline__ uint32_t hash_key_lds(const uint32_t* stg, uint32_t rel, uint32_t n,
                                                 uint32_t seed) {
  uint32_t h = seed ^ (n * kHashM);
  if (n == 0) return h;
  const uint32_t sh = rel & 3u;
  const uint32_t* w0 = stg + (rel >> 2);
  const uint32_t full = n >> 2, r = n & 3u, steps = full + (r ? 1u : 0u);
  for (uint32_t c = 0; c < steps; c += 8) {
    uint32_t w[9];
#pragma unroll
    for (int j = 0; j < 9; j++) w[j] = w0[c + j];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t t = c + j;
      const uint32_t x = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
      if (t < full) {
        h += x;
        h *= kHashM;
        h ^= h >> 16;
      } else if (t == full && r) {
        if (r == 3) h += sext8(x >> 16) << 16;
        if (r >= 2) h += sext8(x >> 8) << 8;
        h += sext8(x);
        h *= kHashM;
        h ^= h >> 24;
      }
    }
  }
  return h;
}

// hash_key_lds when every lane of the wave hashes a key of the same length
// nu (wave-uniform: db_bench keys are all 23 B): the step structure is then
// scalar, straight-line code without per-step lane masks.
__device__ __forceinline__ uint32_t hash_key_lds_uniform(const uint32_t* stg, uint32_t rel,
                                                         uint32_t nu, uint32_t seed) {
  uint32_t h = seed ^ (nu * kHashM);
  if (nu == 0) return h;
  const uint32_t sh = rel & 3u;
  const uint32_t* w = stg + (rel >> 2);
  const uint32_t full = nu >> 2, r = nu & 3u;
  uint32_t lo = w[0];
  uint32_t t = 0;
  for (; t + 4 <= full; t += 4) {  // 16 key bytes per pass
    const uint32_t w1 = w[t + 1], w2 = w[t + 2], w3 = w[t + 3], w4 = w[t + 4];
    h += __builtin_amdgcn_alignbyte(w1, lo, sh);
    h *= kHashM;
    h ^= h >> 16;
    h += __builtin_amdgcn_alignbyte(w2, w1, sh);
    h *= kHashM;
    h ^= h >> 16;
    h += __builtin_amdgcn_alignbyte(w3, w2, sh);
    h *= kHashM;
    h ^= h >> 16;
    h += __builtin_amdgcn_alignbyte(w4, w3, sh);
    h *= kHashM;
    h ^= h >> 16;
    lo = w4;
  }
  for (; t < full; t++) {
    const uint32_t hi = w[t + 1];
    h += __builtin_amdgcn_alignbyte(hi, lo, sh);
    h *= kHashM;
    h ^= h >> 16;
    lo = hi;
  }
  if (r) {
    const uint32_t x = __builtin_amdgcn_alignbyte(w[t + 1], lo, sh);
    // the r tail bytes, each sign-extended, at once: sext8(b) << 8i =
    // (b << 8i) - ((b & 0x80) << (8i + 1)), with wave-uniform masks
    // (5 VALU against 12 for the three-step form)
    const uint32_t m = 0xffffffffu >> (32u - 8u * r), m80 = 0x80808080u & m;
    h += (x & m) - ((x & m80) << 1);
    h *= kHashM;
    h ^= h >> 24;
  }
  return h;
}

// Key i of a batch: [keys + off[i], keys + off[i+1] - strip); empty when the
// key is shorter than strip (ExtractUserKey asserts >= 8, common/dbformat.h:76).
__device__ __forceinline__ void key_extent(const uint8_t* keys, const uint64_t* offs, uint64_t i,
                                           uint32_t strip, uint64_t& s, uint64_t& n) {
  const uint64_t a = offs[i], b = offs[i + 1];
  s = reinterpret_cast<uint64_t>(keys) + a;
  n = b >= a + strip ? b - a - strip : 0;
}

// h % bits for a filter of `bits` bits (util/bloom.cc:58, :84): h is 32-bit and
// bits a size_t, so the result is h itself once bits >= 2^32.  A double multiply
// by the filter's reciprocal gives the quotient to within 2^-23 (h < 2^32,
// bits >= 8), and one +-bits step makes the remainder exact.
struct BitMod {
  double rcp;
  uint32_t d;
  bool big;
};

__device__ __forceinline__ BitMod bit_mod(uint64_t bits) {
  BitMod m;
  m.big = bits > 0xffffffffull;
  m.d = m.big ? 1u : (uint32_t)bits;
  m.rcp = 1.0 / (double)m.d;
  return m;
}

__device__ __forceinline__ uint32_t mod_bits(uint32_t h, const BitMod& m) {
  if (m.big) return h;
  const uint32_t q = (uint32_t)((double)h * m.rcp);
  int64_t r = (int64_t)h - (int64_t)q * (int64_t)m.d;
  if (r < 0) r += m.d;
  else if (r >= (int64_t)m.d) r -= m.d;
  return (uint32_t)r;
}

// n % d for 32-bit n and d by one 64-bit multiply-high chain, with
// M = ceil(2^64 / d) computed once per filter (Lemire, Kaser & Kurz, "Faster
// remainder by direct computation", 2019: exact for every 32-bit n and d).
__device__ __forceinline__ uint64_t fastmod_magic(uint32_t d) { return ~0ull / d + 1; }
__device__ __forceinline__ uint32_t fastmod(uint32_t n, uint64_t M, uint32_t d) {
  const uint64_t low = M * n;  // mod 2^64
  const uint64_t lo = (uint64_t)(uint32_t)low * d, hi = (low >> 32) * d;
  return (uint32_t)((hi + (lo >> 32)) >> 32);  // high 64 bits of low * d
}

// The probe positions of util/bloom.cc:57-61 / :83-87 are h_j mod d with
// h_{j+1} = h_j + delta (mod 2^32).  So after the first one,
//   h_{j+1} mod d = (h_j mod d + s) mod d,
// s = delta mod d, or (delta - 2^32) mod d when h_j + delta carries out of 32
// bits: two remainders per key instead of k, then per probe the add with
// its carry, a select of the step, and p + s reduced as min(p, p - d)
// (unsigned: p - d wraps when p < d).  Needs d < 2^31.  (Round 3 applied the
// carry's correction as a second conditional step: 13 VALU per build probe,
// its LDS address included, against 10 now.)
struct ProbeSeq {
  uint32_t pos, d, h, delta, s0, s1;
  __device__ __forceinline__ void next() {
    const uint32_t hn = h + delta;
    const uint32_t step = hn < h ? s1 : s0;
    h = hn;
    const uint32_t p = pos + step;
    pos = min(p, p - d);
  }
};
// The lookup side's form (key_may_match): the carry's correction applied
// after the step, which needs no second step register (with the
// selected-step form the lookup, then an out-of-line call, spilled 16 B per
// lane per query: 0.49 -> 0.55 ms, profiles/r04/check5/bench_bloom.log).
struct ProbeSeqLookup {
  uint32_t pos, dm, c32, d, h, delta;
  __device__ __forceinline__ void next() {
    const uint32_t hn = h + delta;
    const bool wrap = hn < h;
    h = hn;
    uint32_t p = pos + dm;
    if (p >= d) p -= d;
    if (wrap) p = p >= c32 ? p - c32 : p + (d - c32);
    pos = p;
  }
};
// hm = h mod d, dm = delta mod d, c32 = 2^32 mod d
__device__ __forceinline__ ProbeSeq probe_seq(uint32_t h, uint32_t delta, uint32_t hm, uint32_t dm,
                                              uint32_t c32, uint32_t d) {
  ProbeSeq p;
  p.pos = hm;
  p.d = d;
  p.h = h;
  p.delta = delta;
  p.s0 = dm;
  p.s1 = dm >= c32 ? dm - c32 : dm + (d - c32);
  return p;
}

// Orders one wave's LDS phases (its own ds ops complete in order; this keeps
// the compiler from moving accesses across the phase boundary).
__device__ __forceinline__ void wave_phase() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// LDS bytes [0, n) of the wave's slice -> global [d, d + n), any alignment.
// The aligned middle goes out as dwords (64 lanes x 4 B per instruction); the
// up to 3 + 3 bytes at the ends as byte stores, which leave the bytes of a
// neighbouring filter in the same dword alone.
__device__ __forceinline__ void store_window(uint64_t d, const uint32_t* bm, uint32_t n,
                                             uint32_t lane) {
  const uint8_t* b8 = reinterpret_cast<const uint8_t*>(bm);
  uint32_t head = (4u - ((uint32_t)d & 3u)) & 3u;
  if (head > n) head = n;
  const uint32_t body = (n - head) >> 2;
  const uint32_t tail0 = head + 4 * body;
  if (lane < head) *reinterpret_cast<gu8>(d + lane) = b8[lane];
  if (lane < n - tail0) *reinterpret_cast<gu8>(d + tail0 + lane) = b8[tail0 + lane];
  // source bytes of output dword i: [head + 4i, head + 4i + 4) = words i, i+1
  for (uint32_t i = lane; i < body; i += 64)
    *reinterpret_cast<gu32>(d + head + 4ull * i) = __builtin_amdgcn_alignbyte(bm[i + 1], bm[i], head);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// The bloom hash of this lane's key [s, s + n) (n = 0 on inactive lanes), for
// a whole wave.  When the wave's non-empty keys all lie inside one span that
// fits `avail` bytes of the wave's LDS staging area (64 db_bench keys: 64 x
// 31 B), the span is staged with coalesced 16-B loads -- only 16-B chunks
// that overlap the keys, so never a page the keys do not touch -- and hashed
// from LDS (scalar step structure when all keys have one length); else every
// lane reads its own key's words from global memory.
__device__ __forceinline__ uint32_t wave_hash(uint32_t* stg, uint32_t avail, uint64_t s, uint64_t n,
                                              bool act) {
  const uint32_t lane = threadIdx.x & 63u;
  // the span from the first to the last non-empty key (an empty key's
  // start need not be a readable address)
  const uint64_t nz = __ballot(n > 0);
  const uint32_t fl = nz ? (uint32_t)__builtin_ctzll(nz) : 0u;
  const uint32_t ll = nz ? 63u - (uint32_t)__builtin_clzll(nz) : 0u;
  const uint64_t lo = readlane64(s, fl), hi = readlane64(s + n, ll);
  const uint64_t sbase = lo & ~15ull;
  const bool inside = n == 0 || (s >= lo && s + n <= hi);
  const bool staged = nz != 0 && hi > lo && hi - sbase <= avail && __ballot(!inside) == 0ull;
  if (!staged) return hash_key_batched(s, n, kBloomSeed);
  const uint32_t nch = (uint32_t)((hi - sbase + 15) >> 4);
  for (uint32_t c = lane; c < nch; c += 64)
    *reinterpret_cast<u32x4*>(stg + 4 * c) = *reinterpret_cast<gcu32x4>(sbase + 16ull * c);
  wave_phase();
  const uint32_t rel = act ? (uint32_t)(s - sbase) : 0u;
  const uint32_t n0 = (uint32_t)readlane64(n, fl);
  uint32_t h;
#ifdef LSBM_NO_UNIFORM_HASH  // A/B builds only
  if (false)
#else
  if (__ballot(act && n != n0) == 0ull)  // (inactive lanes' hashes are dropped)
#endif
    h = hash_key_lds_uniform(stg, rel, __builtin_amdgcn_readfirstlane(n0), kBloomSeed);
  else
    h = hash_key_lds(stg, rel, (uint32_t)n, kBloomSeed);
  wave_phase();  // (the next staging writes after these reads)
  return h;
}

// key_offsets[i] and [i + 1] with one 16-byte load (8-byte aligned: gfx950
// global loads take any 4-byte aligned address)
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void load_off2(const uint64_t* ko, uint64_t i, uint64_t& o0, uint64_t& o1) {
  typedef const __attribute__((address_space(1), aligned(8))) u64x2* gp;
  const u64x2 v = *reinterpret_cast<gp>(reinterpret_cast<uint64_t>(ko + i));
  o0 = v.x;
  o1 = v.y;
}

// The build's key staging, pipelined one round ahead: a round's span is
// planned (wave-uniform) and its 16-B chunks loaded into registers -- two per
// lane, spans up to 2 KiB (64 db_bench keys: 1,984 B) -- during the round
// before; the round then writes them to LDS and hashes from there, so no
// round waits for its key words.  Spans that do not fit are hashed from
// global memory (hash_key_batched).
struct SpanPlan {
  uint64_t sbase;  // 16-B aligned start (staged), or a safe 16-B aligned address
  uint32_t nch;    // chunks, 0 when not staged
  uint32_t n0;     // the first non-empty key's length (staged_hash's one-length test)
};

// Wave masks of one compare each, straight from the v_cmp (a __ballot of a
// compound condition compiles to a select and a second compare per lane:
// 2 VALU more per ballot).  Inactive lanes read as 0.
enum : int { kCmpNe = 33, kCmpUgt = 34, kCmpUlt = 36 };
__device__ __forceinline__ uint64_t lanes_ne64(uint64_t a, uint64_t b) { return __builtin_amdgcn_uicmpl(a, b, kCmpNe); }
__device__ __forceinline__ uint64_t lanes_ult64(uint64_t a, uint64_t b) { return __builtin_amdgcn_uicmpl(a, b, kCmpUlt); }
__device__ __forceinline__ uint64_t lanes_ugt64(uint64_t a, uint64_t b) { return __builtin_amdgcn_uicmpl(a, b, kCmpUgt); }
__device__ __forceinline__ uint64_t lanes_ne(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, kCmpNe); }
__device__ __forceinline__ uint64_t lanes_ult(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, kCmpUlt); }
// lanes [0, m) of the wave (m wave-uniform): scalar only
__device__ __forceinline__ uint64_t first_lanes(uint64_t m) { return m >= 64 ? ~0ull : (1ull << m) - 1ull; }

__device__ __forceinline__ SpanPlan plan_span(uint64_t s, uint64_t n, uint32_t cap, uint64_t safe) {
  const uint64_t nz = lanes_ne64(n, 0);
  const uint32_t fl = nz ? (uint32_t)__builtin_ctzll(nz) : 0u;
  const uint32_t ll = nz ? 63u - (uint32_t)__builtin_clzll(nz) : 0u;
  const uint64_t lo = readlane64(s, fl), hi = readlane64(s + n, ll);
  const uint64_t sbase = lo & ~15ull;
  // a non-empty key outside [lo, hi)
  const uint64_t outside = nz & (lanes_ult64(s, lo) | lanes_ugt64(s + n, hi));
  // lo < hi <= lo + 2048 iff hi - lo - 1 < 2048 (64-bit), and then the span
  // [sbase, hi) fits 32 bits: scalar compares only (a 64-bit compare of two
  // wave-uniform values goes to the VALU)
  const uint64_t d1 = hi - lo - 1u;
  const uint32_t span = (uint32_t)d1 + 1u + ((uint32_t)lo & 15u);
  const bool staged = nz != 0 && (uint32_t)(d1 >> 32) == 0u && (uint32_t)d1 < 2048u && span <= 2048u && span <= cap &&
                      outside == 0ull;
  SpanPlan p;
  p.sbase = staged ? sbase : safe;
  p.nch = staged ? (span + 15u) >> 4 : 0u;
  p.n0 = (uint32_t)readlane64(n, fl);
  return p;
}

// Every lane loads (unconditionally, from a readable chunk) so that the loads
// in flight are the same on every path.
__device__ __forceinline__ void fetch_span(const SpanPlan& p, u32x4& c0, u32x4& c1) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t a0 = lane < p.nch ? p.sbase + 16ull * lane : p.sbase;
  const uint64_t a1 = lane + 64u < p.nch ? p.sbase + 16ull * (lane + 64u) : p.sbase;
  c0 = *reinterpret_cast<gcu32x4>(a0);
  c1 = *reinterpret_cast<gcu32x4>(a1);
}

// (actm: the wave's active lanes, act = bit lane of actm)
__device__ __forceinline__ uint32_t staged_hash(uint32_t* stg, const SpanPlan& p, u32x4 c0, u32x4 c1,
                                                uint64_t s, uint64_t n, bool act, uint64_t actm) {
  const uint32_t lane = threadIdx.x & 63u;
  if (p.nch == 0) return hash_key_batched(s, n, kBloomSeed);
  if (lane < p.nch) *reinterpret_cast<u32x4*>(stg + 4 * lane) = c0;
  if (lane + 64u < p.nch) *reinterpret_cast<u32x4*>(stg + 4 * (lane + 64u)) = c1;
  wave_phase();
  const uint32_t rel = act ? (uint32_t)(s - p.sbase) : 0u;
  uint32_t h;
  // (staged: every key is inside the span, n < 2 KiB)
  if ((lanes_ne((uint32_t)n, p.n0) & actm) == 0ull)
    h = hash_key_lds_uniform(stg, rel, p.n0, kBloomSeed);
  else
    h = hash_key_lds(stg, rel, (uint32_t)n, kBloomSeed);
  wave_phase();  // (the next round's staging writes after these reads)
  return h;
}

// One filter, keys [k0, k1), written to out + fo, in LDS windows of
// kBloomWindowBytes (the path for filters a packed batch cannot hold).
__device__ void build_one(const BloomBuildArgs& a, uint64_t k0, uint64_t k1, uint64_t fo,
                          uint32_t* bm, uint32_t lane) {
  // util/bloom.cc:39-46: bits = max(64, n * bits_per_key), rounded up to bytes
  const uint64_t nk = k1 > k0 ? k1 - k0 : 0;
  uint64_t bits = nk * a.bits_per_key;
  if (bits < 64) bits = 64;
  const uint64_t bytes = (bits + 7) / 8;
  const BitMod m = bit_mod(bytes * 8);
  const uint64_t dst = reinterpret_cast<uint64_t>(a.out) + fo;
  for (uint64_t win = 0; win < bytes; win += kBloomWindowBytes) {
    const uint32_t wbytes =
        (uint32_t)(bytes - win < kBloomWindowBytes ? bytes - win : kBloomWindowBytes);
    const uint64_t bit0 = win * 8, nbits = (uint64_t)wbytes * 8;
    for (uint32_t i = lane; i <= wbytes / 4; i += 64) bm[i] = 0;  // + 1 pad word
    wave_phase();
    // util/bloom.cc:52-62: double hashing, delta = h rotated right 17
    for (uint64_t i = k0 + lane; i < k1; i += 64) {
      uint64_t s, n;
      key_extent(a.keys, a.key_offsets, i, a.strip, s, n);
      uint32_t h = hash_key(s, n, kBloomSeed);
      const uint32_t delta = (h >> 17) | (h << 15);
      for (uint32_t j = 0; j < a.k; j++) {
        const uint64_t rel = (uint64_t)mod_bits(h, m) - bit0;  // wraps below the window
        if (rel < nbits) atomicOr(&bm[rel >> 5], 1u << (rel & 31u));
        h += delta;
      }
    }
    wave_phase();
    store_window(dst + win, bm, wbytes, lane);
    wave_phase();
  }
  if (lane == 0) *reinterpret_cast<gu8>(dst + bytes) = (uint8_t)a.k;  // :50
}

// A wave takes kBloomGroup consecutive filters at a time.  When their keys
// are contiguous and their bit arrays fit the wave's LDS region (db_bench: 32 x
// 84 B), the keys of all of them are spread over the 64 lanes round by round
// (a 33-key filter would leave half the lanes idle at one filter per wave):
// each lane finds its key's filter by a binary search over the group's first
// keys (held one per lane, read with bpermute), takes that filter's bit-array
// base, size and remainder constants from the filter's LDS slot, and sets its k
// bits with ds_or_b32 in the filter's part of the LDS image; every filter
// leaves LDS once.  The round's key words are staged in the region's free
// tail (wave_hash).  Otherwise the group's filters go one by one through
// build_one.
// LDS byte address of p (a pointer into __shared__ memory), and the LDS word
// holding bit b (an LDS bit address) or-ed with v
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
  return (uint32_t)(uintptr_t)(const lds_u32*)p;
}
__device__ __forceinline__ void lds_or(uint32_t b, uint32_t v) {
  lds_u32* w = (lds_u32*)(uintptr_t)((b >> 3) & ~3u);
  (void)__hip_atomic_fetch_or(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#ifndef LSBM_BUILD_WAVES_PER_EU  // (A/B builds override)
#define LSBM_BUILD_WAVES_PER_EU 7
#endif
// 7 waves per SIMD (<= 72 VGPRs): the grid is sized for 7 workgroups per CU
// (A/B: 6 -> 0.372 ms, 7 -> 0.358 ms, 8 -> 0.419 ms with scratch spills)
__global__ __launch_bounds__(kBloomThreads) __attribute__((amdgpu_waves_per_eu(LSBM_BUILD_WAVES_PER_EU)))
void bloom_build_kernel(BloomBuildArgs a) {
  // (rows of kBloomRegionWords: 16-B aligned, for the staging area's b128 writes)
  __shared__ __attribute__((aligned(16))) uint32_t lds[kBloomWaves][kBloomRegionWords];
  // the group's filter constants, one slot per filter: its first bit as an LDS bit address, bits d,
  // fastmod magic (lo, hi); and 2^32 mod d.  (Read by index rather than with
  // bpermute from the filter's lane: 5 fewer VGPRs live across the rounds,
  // 0.354 -> 0.348 ms, profiles/r02/bloom/ab_slots.log.)
  __shared__ __attribute__((aligned(16))) uint4 slots[kBloomWaves][kBloomGroup];
  __shared__ uint32_t slot_c32[kBloomWaves][kBloomGroup];
  static_assert(LSBM_BUILD_WAVES_PER_EU * (sizeof(lds) + sizeof(slots) + sizeof(slot_c32)) <= 160u * 1024u,
                "the build grid's workgroups per CU must fit one CU's LDS");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* bm = lds[wv];
  // Waves stride over groups of kBloomGroup consecutive filters.  (Tried:
  // contiguous per-wave ranges, and a group size chosen so that every wave
  // gets the same number of groups: 4% slower both)
  const uint64_t nwaves = (uint64_t)gridDim.x * kBloomWaves;
  const uint64_t n_groups = (a.n_filters + kBloomGroup - 1) / kBloomGroup;
  const uint64_t kbase = reinterpret_cast<uint64_t>(a.keys);
  // lane t < g: filter f0 + t.  A group's filter table entries are loaded
  // while the group before writes its filters out.
  uint64_t mk0 = 0, mk1 = 0, mfo = 0;
  auto load_meta = [&](uint64_t grp) {
    const uint64_t f0 = grp * kBloomGroup;
    mk0 = mk1 = mfo = 0;
    if (grp < n_groups && lane < a.n_filters - f0 && lane < kBloomGroup) {
      mk0 = a.filter_first[f0 + lane];
      mk1 = a.filter_first[f0 + lane + 1];
      mfo = a.filter_out[f0 + lane];
    }
  };
  load_meta((uint64_t)blockIdx.x * kBloomWaves + wv);
  for (uint64_t grp = (uint64_t)blockIdx.x * kBloomWaves + wv; grp < n_groups; grp += nwaves) {
    const uint64_t f0 = grp * kBloomGroup;
    const uint32_t g = (uint32_t)(a.n_filters - f0 < kBloomGroup ? a.n_filters - f0 : kBloomGroup);
    uint64_t k0 = 0, k1 = 0, fo = 0, bytes = 0;
    k0 = mk0;  // (0 past the group)
    k1 = mk1;
    fo = mfo;
    if (lane < g) {
      uint64_t bits = (k1 > k0 ? k1 - k0 : 0) * a.bits_per_key;
      if (bits < 64) bits = 64;
      bytes = (bits + 7) / 8;
    }
    // LDS words of each filter (+ 1 pad word for the funnel-shifted store)
    const uint64_t words = lane < g ? (bytes + 3) / 4 + 1 : 0;
    uint64_t incl = words;
#pragma unroll
    for (uint32_t d = 1; d < kBloomGroup; d <<= 1) {
      const uint64_t t = __shfl_up(incl, d);
      if (lane >= d) incl += t;
    }
    const uint64_t kb0 = readlane64(k0, 0), kb1 = readlane64(k1, g - 1);
    const uint64_t next0 = __shfl_down(k0, 1);
    const bool contiguous = lane >= g || (k1 >= k0 && (lane == g - 1 || next0 == k1));
    // Dense layout: when the group's filters follow each other in the output
    // (each one's bits, then its k byte: FilterBlockBuilder's result_), LDS
    // holds the output image itself, at the destination's byte alignment, and
    // leaves as one run of dword stores (bytes at the two ends).  Otherwise
    // each filter sits at a dword boundary with a pad word and leaves alone.
    const uint64_t fo_next = __shfl_down(fo, 1);
    const bool out_next = lane + 1 >= g || fo_next == fo + bytes + 1;
    const uint64_t fo0 = readlane64(fo, 0);
    const uint64_t dst0 = reinterpret_cast<uint64_t>(a.out) + fo0;
    const uint32_t gsh = (uint32_t)dst0 & 3u;
    const uint64_t span = readlane64(fo + bytes + 1, g - 1) - fo0;  // (dense: the group's output bytes)
    const bool dense = __ballot(!out_next) == 0 && span < (1ull << 20);
    const uint64_t total = dense ? (gsh + span + 3) / 4 : readlane64(incl, kBloomGroup - 1);
    const bool packed = __ballot(!contiguous) == 0 && total <= kBloomRegionWords &&
                        kb1 >= kb0 && kb1 - kb0 < (1ull << 31);
    if (!packed) {
      load_meta(grp + nwaves);
      for (uint32_t j = 0; j < g; j++)
        build_one(a, readlane64(k0, j), readlane64(k1, j), readlane64(fo, j), bm, lane);
      continue;
    }
    const uint32_t nkeys = (uint32_t)(kb1 - kb0);
    const uint64_t* ko = a.key_offsets + kb0;
    const uint64_t safe = reinterpret_cast<uint64_t>(ko) & ~15ull;  // a readable 16-B chunk
    // Key offsets are loaded two rounds ahead and key words (staged) one
    // round ahead: round r holds the offsets of rounds r and r + 1.
    uint64_t oa0 = 0, oa1 = 0, ob0 = 0, ob1 = 0;
    if (lane < nkeys) load_off2(ko, lane, oa0, oa1);
    if (lane + 64u < nkeys) load_off2(ko, lane + 64, ob0, ob1);
    // filter t's constants, from lane t, into slot t: LDS bit base, bits d,
    // fastmod magic, 2^32 mod d; and (in lane t) its first key relative to the group's (non-decreasing;
    // ~0 past the group, so that a search never selects those lanes)
    const uint32_t base_t = (uint32_t)(incl - words);  // (sparse layout: word base)
    const uint32_t byte_t = dense ? gsh + (uint32_t)(fo - fo0) : 4u * base_t;
    if (lane < kBloomGroup) {
      const uint32_t d_t = lane < g ? (uint32_t)(bytes * 8) : 64u;
      const uint64_t m_t = fastmod_magic(d_t);
      const uint32_t c = fastmod(0xffffffffu, m_t, d_t) + 1;
      // (the bit base counts from LDS address 0: a probe's word address is
      // then (b >> 3) & ~3 with no region base added, one VALU per probe
      // less: 0.300 -> 0.295-0.298 ms, profiles/r04/check11/build_*.log)
      slots[wv][lane] = make_uint4(8u * (lds_addr(bm) + byte_t), d_t, (uint32_t)m_t, (uint32_t)(m_t >> 32));
      slot_c32[wv][lane] = c == d_t ? 0u : c;
    }
    const uint32_t st_t = lane < g ? (uint32_t)(k0 - kb0) : 0xffffffffu;
    for (uint32_t i = lane; i < (uint32_t)total; i += 64) bm[i] = 0;
    wave_phase();
    if (dense && lane < g)  // each filter's k byte (util/bloom.cc:50), after its bits
      reinterpret_cast<uint8_t*>(bm)[byte_t + (uint32_t)bytes] = (uint8_t)a.k;
    wave_phase();
    // the staging area: the region's free tail, less 48 B that a key's hash
    // may read past the span (none at all when the filters fill the region)
    const uint32_t used = (uint32_t)((total + 3u) & ~3ull) * 4u;
    uint32_t* stg = bm + used / 4u;
    const uint32_t avail = used + 48u < kBloomRegionWords * 4u ? kBloomRegionWords * 4u - used - 48u : 0u;
    // A round's key (start, length) is computed once, with its span plan a
    // round ahead, and carried to the round.
    // A round's key (start, length) is computed once, with its span plan a
    // round ahead, and carried to the round.  (Tried: two register sets
    // alternating between rounds, which drops the 6 v_mov_b64 a round that
    // move the next round's set into the current one: no faster, twice the
    // code; profiles/r04/check26/.)
    SpanPlan plan;
    u32x4 ch0, ch1;
    uint64_t ks = 0, kn = 0;
    {
      const bool act = lane < nkeys;
      kn = act && oa1 >= oa0 + a.strip ? oa1 - oa0 - a.strip : 0;  // key_extent
      ks = kbase + oa0;
      plan = plan_span(ks, kn, avail, safe);
      fetch_span(plan, ch0, ch1);
    }
    uint32_t c0 = 0;  // filters starting before the round
    for (uint32_t r0 = 0; r0 < nkeys; r0 += 64) {  // wave-uniform rounds
      const uint32_t r = r0 + lane;
      const uint64_t actm = first_lanes(nkeys - r0);
      const bool act = r < nkeys;
      // the last filter of the group whose first key is <= r (empty filters
      // share their successor's first key and are passed over): the filters
      // starting before the round, plus those starting inside it at or before
      // r -- a wave-uniform handful (~2 of 33-key filters per 64-key round),
      // each read with readlane.  (Round 3: a 5-step binary search, a chain
      // of dependent ds_bpermute round trips every round.)  st_t is ~0 past
      // the group: one compare counts the group's filters.
      const uint32_t c1 = (uint32_t)__builtin_popcountll(lanes_ult(st_t, r0 + 64u));
      uint32_t cnt = c0;
      for (uint32_t q = c0; q < c1; q++)
        cnt += (uint32_t)__builtin_amdgcn_readlane((int)st_t, (int)q) <= r ? 1u : 0u;
      c0 = c1;
      const uint32_t j = cnt - 1u;  // (filter 0 starts at key 0: cnt >= 1)
      const uint4 sl = slots[wv][j];
      const uint32_t bbase = sl.x, d = sl.y;
      const uint64_t M = ((uint64_t)sl.w << 32) | sl.z;
      const uint32_t c32 = slot_c32[wv][j];
      const uint64_t s = ks, n = kn;
      // this round's chunks into LDS, then the next round's plan and loads
      const SpanPlan cur = plan;
      const u32x4 cc0 = ch0, cc1 = ch1;
      {
        const bool act1 = r + 64u < nkeys;
        kn = act1 && ob1 >= ob0 + a.strip ? ob1 - ob0 - a.strip : 0;
        ks = kbase + ob0;
        plan = plan_span(ks, kn, avail, safe);
        fetch_span(plan, ch0, ch1);
        if (r + 128u < nkeys) load_off2(ko, r + 128, ob0, ob1);
      }
      const uint32_t h = staged_hash(stg, cur, cc0, cc1, s, n, act, actm);
      if (!act) continue;
      const uint32_t delta = (h >> 17) | (h << 15);  // util/bloom.cc:56-61
      ProbeSeq ps = probe_seq(h, delta, fastmod(h, M, d), fastmod(delta, M, d), c32, d);
#ifdef LSBM_PROBE_UNROLL  // A/B builds only
#pragma unroll LSBM_PROBE_UNROLL
#endif
#ifdef LSBM_DIAG_NO_PROBE_WRITES  // (diagnostic A/B builds only: wrong filters)
      uint32_t acc = 0;
      for (uint32_t q = 0; q < a.k; q++) {
        acc ^= bbase + ps.pos;
        ps.next();
      }
      if (acc == 0xffffffffu) bm[0] = acc;
#else
      for (uint32_t q = 0; q < a.k; q++) {
        const uint32_t b = bbase + ps.pos;
        lds_or(b, 1u << (b & 31u));
        ps.next();
      }
#endif
    }
    load_meta(grp + nwaves);
    wave_phase();
    if (dense) {
      // LDS byte x <-> global byte dst0 - gsh + x, for x in [gsh, gsh + span):
      // whole dwords as dword stores, the partial first / last dword as bytes
      // (they share a dword with a neighbouring group's output)
      const uint32_t end = gsh + (uint32_t)span;
      const uint64_t gbase = dst0 - gsh;
      for (uint32_t i = lane; i < (uint32_t)total; i += 64) {
        if (4 * i >= gsh && 4 * i + 4 <= end) {
          *reinterpret_cast<gu32>(gbase + 4ull * i) = bm[i];
        } else {
          const uint32_t v = bm[i];
          for (uint32_t q = 0; q < 4; q++)
            if (4 * i + q >= gsh && 4 * i + q < end) *reinterpret_cast<gu8>(gbase + 4ull * i + q) = (uint8_t)(v >> (8 * q));
        }
      }
    } else {
      for (uint32_t j = 0; j < g; j++) {
        const uint64_t dst = reinterpret_cast<uint64_t>(a.out) + readlane64(fo, j);
        const uint32_t nb = (uint32_t)readlane64(bytes, j);
        store_window(dst, bm + __builtin_amdgcn_readlane(base_t, j), nb, lane);
        if (lane == 0) *reinterpret_cast<gu8>(dst + nb) = (uint8_t)a.k;  // :50
      }
    }
    wave_phase();
  }
}

__device__ __forceinline__ uint64_t load_le32(uint64_t p) {  // DecodeFixed32, any alignment
  const gcu8 b = reinterpret_cast<gcu8>(p);
  return (uint64_t)b[0] | ((uint64_t)b[1] << 8) | ((uint64_t)b[2] << 16) | ((uint64_t)b[3] << 24);
}

// util/bloom.cc:65-89 on the filter [f, f + len).  Inlined: as a call, its
// entry waited for every load the probe kernel had in flight (the next
// rounds' key words and offsets); inlined the kernels still fit 80 / 95 VGPRs
// (6 / 5 waves per SIMD): 0.449 -> 0.441 ms one filter per query, 0.535 ->
// 0.511 ms through filter blocks (profiles/r04/check30/).
__device__ __forceinline__ bool key_may_match(uint64_t f, uint64_t len, uint32_t h, uint64_t k_use) {
  if (len < 2) return false;
  const uint64_t bits = (len - 1) * 8;
  const BitMod m = bit_mod(bits);
  const uint32_t delta = (h >> 17) | (h << 15);
  const bool inc = bits < (1ull << 31);  // ProbeSeq's range; else a remainder per probe
  ProbeSeqLookup ps{0, 0, 0, (uint32_t)bits, h, delta};
  if (inc) {
    ps.pos = mod_bits(h, m);
    ps.dm = mod_bits(delta, m);
    const uint32_t c = mod_bits(0xffffffffu, m) + 1;  // 2^32 mod bits
    ps.c32 = c == ps.d ? 0 : c;
  }
  // The reference stops at the first clear bit (:85); the answer is the same
  // if a chunk of up to 16 probe bytes (all inside this filter) is requested
  // at once and tested together: one round trip instead of up to k.  The
  // probe positions do not depend on the filter's stored k, so the first
  // chunk (min(k_use, 16) probes) is requested together with the k byte:
  // one round trip less per lookup (those past k are loaded and ignored).
  const uint32_t k0n = k_use < 16 ? (uint32_t)k_use : 16u;
#ifdef LSBM_DIAG_NO_FILTER_LOADS  // (diagnostic A/B builds only: what the filter round trip costs)
  return ((ps.pos ^ ps.dm ^ (uint32_t)f) & 1u) != 0;
#endif
  const uint8_t kb = *reinterpret_cast<gcu8>(f + len - 1);
  uint32_t v[16], bit[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    bit[j] = 0u;
    v[j] = 0u;
    if ((uint32_t)j < k0n) {  // (k_use is the same in every lane)
      const uint32_t bitpos = inc ? ps.pos : mod_bits(ps.h, m);
      bit[j] = 1u << (bitpos & 7u);
      v[j] = *reinterpret_cast<gcu8>(f + (bitpos >> 3));
      if (inc) ps.next();
      else ps.h += delta;
    }
  }
  // `array[len-1] > k_use_`: a signed char converted to size_t
  const uint64_t stored = (uint64_t)(int64_t)(int8_t)kb;
  const uint64_t k = stored > k_use ? k_use : stored;
  if (k > 30) return true;
  bool all = true;
#pragma unroll
  for (int j = 0; j < 16; j++) all &= (uint32_t)j >= k || (v[j] & bit[j]) == bit[j];
  if (!all) return false;
  for (uint32_t j0 = k0n; j0 < (uint32_t)k; j0 += 16) {  // (k_use > 16 only)
#pragma unroll
    for (int j = 0; j < 16; j++) {
      bit[j] = 0u;
      v[j] = 0u;
      if (j0 + j < (uint32_t)k) {
        const uint32_t bitpos = inc ? ps.pos : mod_bits(ps.h, m);
        bit[j] = 1u << (bitpos & 7u);
        v[j] = *reinterpret_cast<gcu8>(f + (bitpos >> 3));
        if (inc) ps.next();
        else ps.h += delta;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j++) all &= (v[j] & bit[j]) == bit[j];
    if (!all) return false;
  }
  return true;
}

constexpr uint32_t kProbeStageWords = 576;  // a wave's key staging area (64 x 31-B keys + slack)

// One instantiation per mode (the other mode's code dropped).  The
// one-filter-per-query probe is held to 6 waves per SIMD (<= 80 VGPRs, a few
// spilled outside the probe loop): 0.504 -> 0.491 ms against the 5 waves its
// 90 VGPRs allow; the filter-block probe, whose spills would sit in its
// offset-array lookups, ran 0.61 -> 0.82 ms under the same bound and keeps
// its registers (profiles/r02/bloom/ab_probe_pipelined.log).
#ifndef LSBM_PROBE_WAVES_PER_EU  // (A/B builds override)
#define LSBM_PROBE_WAVES_PER_EU 6
#endif
#ifndef LSBM_PROBE_BLOCK_WAVES_PER_EU  // (A/B builds override)
#define LSBM_PROBE_BLOCK_WAVES_PER_EU 5  // (<= 96 VGPRs: the pipelined lookups fit without spills)
#endif
#ifndef LSBM_BLOCK_AHEAD  // (A/B builds: 0 = each round's filter-block lookup after its own hash)
#define LSBM_BLOCK_AHEAD 1
#endif

// FilterBlockReader::KeyMayMatch's filter lookup (table/filter_block.cc:78-109)
// without the key: which filter of block [c, c + size) a data block at offset
// doff uses.  kProbe: probe [f, f + len); kMay: "errors are treated as
// potential matches"; kNo: an empty filter matches nothing.  base_lg is a
// size_t loaded from a char, the shift count taken mod 64 (x86-64).
enum : uint32_t { kBlkProbe = 0, kBlkMay = 1, kBlkNo = 2 };
struct BlockTrailer {  // the block's last 5 bytes: the offset array's position and base_lg
  uint32_t lg, lw;
};
__device__ __forceinline__ BlockTrailer block_trailer(uint64_t c, uint64_t size, uint64_t dummy) {
  const bool ok = size >= 5;
  BlockTrailer t;
  t.lg = *reinterpret_cast<gcu8>(ok ? c + size - 1 : dummy);
  t.lw = (uint32_t)load_le32(ok ? c + size - 5 : dummy);
  return t;
}
// the offset array entry's address (or dummy, with *state = kBlkMay: no entry)
__device__ __forceinline__ uint64_t block_entry(uint64_t c, uint64_t size, uint64_t doff, BlockTrailer t,
                                                uint64_t dummy, uint32_t* state) {
  const uint64_t base_lg = (uint64_t)(int64_t)(int8_t)(uint8_t)t.lg;
  const uint64_t last_word = t.lw;
  bool ok = size >= 5 && last_word <= size - 5;
  const uint64_t num = ok ? (size - 5 - last_word) / 4 : 0;
  const uint64_t index = doff >> (base_lg & 63u);
  ok = ok && index < num;
  *state = ok ? kBlkProbe : kBlkMay;
  return ok ? c + last_word + index * 4 : dummy;
}
template <uint32_t kMode>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(kMode == kProbeFilter ? LSBM_PROBE_WAVES_PER_EU : LSBM_PROBE_BLOCK_WAVES_PER_EU)))
void bloom_probe_kernel(BloomProbeArgs a) {
  a.mode = kMode;  // compile-time: the other mode's code is dropped
  __shared__ __attribute__((aligned(16))) uint32_t stage[4][kProbeStageWords];
  uint32_t* stg = stage[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t hits = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // wave-uniform rounds of 64 consecutive queries (the hash is a wave operation)
#ifndef LSBM_PROBE_NO_PIPELINE  // A/B builds only
  // Pipelined like the build: a round's key offsets are loaded two rounds
  // ahead and its staged key words (16-B chunks in registers) one round
  // ahead, so no round waits for its keys.
  const uint64_t kbase = reinterpret_cast<uint64_t>(a.keys);
  const uint64_t safe = reinterpret_cast<uint64_t>(a.key_offsets) & ~15ull;  // a readable 16-B chunk
  const uint32_t avail = kProbeStageWords * 4u - 48u;
  const uint64_t q00 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  uint64_t oa0 = 0, oa1 = 0, ob0 = 0, ob1 = 0;
  if (q00 + lane < a.n) load_off2(a.key_offsets, q00 + lane, oa0, oa1);
  if (q00 + stride + lane < a.n) load_off2(a.key_offsets, q00 + stride + lane, ob0, ob1);
  // (a round's key start and length: computed once, with its plan, and carried)
  SpanPlan plan;
  u32x4 ch0, ch1;
  uint64_t ksn = 0, knn = 0;
  {
    const bool act = q00 + lane < a.n;
    knn = act && oa1 >= oa0 + a.strip ? oa1 - oa0 - a.strip : 0;  // key_extent
    ksn = kbase + oa0;
    plan = plan_span(ksn, knn, avail, safe);
    fetch_span(plan, ch0, ch1);
  }
  // Filter blocks, LSBM_BLOCK_AHEAD: a round's filter lookup does not depend
  // on its keys, so it runs ahead of them as a pipeline -- the handle two
  // rounds ahead, the block's trailer one round ahead before the hash, the
  // offset-array entry one round ahead after it -- and a round's probes wait
  // only for its hash (round 3: handle, trailer and entry one after another
  // behind the hash).
  constexpr bool kAhead = kMode == kProbeFilterBlock && LSBM_BLOCK_AHEAD;
  const uint64_t fbase = reinterpret_cast<uint64_t>(a.base);
  const uint64_t dummy = reinterpret_cast<uint64_t>(a.handles);  // (16 readable bytes)
  uint64_t hc1 = 0, hs1 = 0, hd1 = 0;  // round r + 1's handle and data offset
  uint64_t bf = 0;                     // round r's filter [bf, bf + blen), or its verdict bst
  uint32_t blen = 0, bst = kBlkMay;
  if constexpr (kAhead) {
    const uint64_t q0q = q00 + lane < a.n ? q00 + lane : 0;
    const uint64_t c0 = fbase + a.handles[2 * q0q], s0 = a.handles[2 * q0q + 1], d0 = a.data_offsets[q0q];
    const BlockTrailer t0 = block_trailer(c0, s0, dummy);
    const uint64_t e0 = block_entry(c0, s0, d0, t0, dummy, &bst);
    const uint32_t st0 = (uint32_t)load_le32(e0), li0 = (uint32_t)load_le32(e0 + 4);
    if (bst == kBlkProbe) {
      bst = st0 <= li0 && li0 <= t0.lw ? kBlkProbe : st0 == li0 ? kBlkNo : kBlkMay;
      bf = c0 + st0;
      blen = li0 - st0;
    }
    const uint64_t q1q = q00 + stride + lane < a.n ? q00 + stride + lane : 0;
    hc1 = fbase + a.handles[2 * q1q];
    hs1 = a.handles[2 * q1q + 1];
    hd1 = a.data_offsets[q1q];
  }
  for (uint64_t q0 = q00; q0 < a.n; q0 += stride) {
    const uint64_t q = q0 + lane;
    const bool act = q < a.n;
    const uint64_t actm = first_lanes(a.n - q0);
    const uint64_t ks = ksn, kn = knn;
    // the filter handle (and data offset) do not depend on the hash: requested
    // before it (the hash's LDS fences would otherwise hold them back)
    uint64_t c = 0, size = 0, doff = 0;
    uint64_t hc2 = 0, hs2 = 0, hd2 = 0;
    BlockTrailer t1 = {0, 0};
    if constexpr (kAhead) {
      const uint64_t q2 = q + 2 * stride < a.n ? q + 2 * stride : 0;  // round r + 2's handle
      hc2 = fbase + a.handles[2 * q2];
      hs2 = a.handles[2 * q2 + 1];
      hd2 = a.data_offsets[q2];
      t1 = block_trailer(hc1, hs1, dummy);  // round r + 1's trailer
    } else {
      const uint64_t qq = act ? q : 0;
      c = fbase + a.handles[2 * qq];
      size = a.handles[2 * qq + 1];
      doff = a.mode == kProbeFilter ? 0 : a.data_offsets[qq];
    }
    // this round's chunks go to LDS; the next round's plan and loads go out
    const SpanPlan cur = plan;
    const u32x4 cc0 = ch0, cc1 = ch1;
    {
      const bool act1 = q + stride < a.n;
      knn = act1 && ob1 >= ob0 + a.strip ? ob1 - ob0 - a.strip : 0;
      ksn = kbase + ob0;
      plan = plan_span(ksn, knn, avail, safe);
      fetch_span(plan, ch0, ch1);
      if (q + 2 * stride < a.n) load_off2(a.key_offsets, q + 2 * stride, ob0, ob1);
    }
    const uint32_t h = staged_hash(stg, cur, cc0, cc1, ks, kn, act, actm);
    if constexpr (kAhead) {
      // round r + 1's offset-array entry, then round r's probes
      uint32_t st1;
      const uint64_t e1 = block_entry(hc1, hs1, hd1, t1, dummy, &st1);
      const uint32_t start1 = (uint32_t)load_le32(e1), limit1 = (uint32_t)load_le32(e1 + 4);
      if (act) {
        const bool may = bst == kBlkProbe ? key_may_match(bf, blen, h, a.k_use) : bst == kBlkMay;
        a.may[q] = may ? 1 : 0;
        hits += may ? 1u : 0u;
      }
      if (st1 == kBlkProbe)
        st1 = start1 <= limit1 && limit1 <= t1.lw ? kBlkProbe : start1 == limit1 ? kBlkNo : kBlkMay;
      bst = st1;
      bf = hc1 + start1;
      blen = limit1 - start1;
      hc1 = hc2;
      hs1 = hs2;
      hd1 = hd2;
      continue;
    }
    if (!act) continue;
#else
    uint64_t c, size, doff;
  for (uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); q0 < a.n; q0 += stride) {
    const uint64_t q = q0 + lane;
    const bool act = q < a.n;
    uint64_t ks = reinterpret_cast<uint64_t>(a.keys), kn = 0;
    if (act) key_extent(a.keys, a.key_offsets, q, a.strip, ks, kn);
    const uint64_t qq = act ? q : 0;
    c = reinterpret_cast<uint64_t>(a.base) + a.handles[2 * qq];
    size = a.handles[2 * qq + 1];
    doff = a.mode == kProbeFilter ? 0 : a.data_offsets[qq];
    const uint32_t h = wave_hash(stg, kProbeStageWords * 4u - 48u, ks, kn, act);
    if (!act) continue;
#endif
    bool may;
    if (a.mode == kProbeFilter) {
      may = key_may_match(c, size, h, a.k_use);
    } else {
      // FilterBlockReader (table/filter_block.cc:78-109): "errors are treated
      // as potential matches"; base_lg is a size_t loaded from a char, and the
      // shift count is taken mod 64 as on the x86-64 reference build
      may = true;
      if (size >= 5) {
        const uint64_t base_lg = (uint64_t)(int64_t)(int8_t)*reinterpret_cast<gcu8>(c + size - 1);
        const uint64_t last_word = load_le32(c + size - 5);
        if (last_word <= size - 5) {
          const uint64_t num = (size - 5 - last_word) / 4;
          const uint64_t index = doff >> (base_lg & 63u);
          if (index < num) {
            const uint64_t start = load_le32(c + last_word + index * 4);
            const uint64_t limit = load_le32(c + last_word + index * 4 + 4);
            if (start <= limit && limit <= last_word)
              may = key_may_match(c + start, limit - start, h, a.k_use);
            else if (start == limit)
              may = false;  // an empty filter matches nothing
          }
        }
      }
    }
    a.may[q] = may ? 1 : 0;
    hits += may ? 1u : 0u;
  }
  if (a.n_may) {  // one atomic per wave
    for (int o = 32; o; o >>= 1) hits += (uint32_t)__shfl_xor((int)hits, o);
    if (lane == 0 && hits) atomicAdd(a.n_may, hits);
  }
}

}  // namespace

// ---- host-callable launchers (used by bloom_engine.cc) ----
hipError_t launch_bloom_build(const BloomBuildArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(bloom_build_kernel, dim3(grid), dim3(kBloomThreads), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_bloom_probe(const BloomProbeArgs& a, int grid, hipStream_t stream) {
  if (a.mode == kProbeFilter)
    hipLaunchKernelGGL(bloom_probe_kernel<kProbeFilter>, dim3(grid), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(bloom_probe_kernel<kProbeFilterBlock>, dim3(grid), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// Workgroups of each kernel resident per CU (registers, LDS): grid-stride
// launches size their grids to fill the chip exactly once.
int bloom_build_blocks_per_cu() {
#ifdef LSBM_BUILD_WGS  // A/B builds only
  return LSBM_BUILD_WGS;
#endif
  // = LSBM_BUILD_WAVES_PER_EU (one wave per SIMD per workgroup).  Measured:
  // without the waves-per-EU bound the kernel took 79-95 VGPRs and only 6
  // workgroups fitted although the occupancy query reported 7; a 7-per-CU
  // grid then ran 30% slower, as a second batch.
  return LSBM_BUILD_WAVES_PER_EU;
  static const int v = [] {
    int b = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, bloom_build_kernel, kBloomThreads, 0) ==
                       hipSuccess && b > 0 ? b : 4;
  }();
  return v;
}

int bloom_probe_blocks_per_cu(uint32_t mode) {
#ifdef LSBM_PROBE_WGS  // A/B builds only
  return LSBM_PROBE_WGS;
#endif
  auto query = [](const void* k) {
    int b = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0) == hipSuccess && b > 0 ? b : 4;
  };
  static const int v0 = query(reinterpret_cast<const void*>(bloom_probe_kernel<kProbeFilter>));
  static const int v1 = query(reinterpret_cast<const void*>(bloom_probe_kernel<kProbeFilterBlock>));
  return mode == kProbeFilter ? v0 : v1;
}

}  // namespace lsbm
