// crc32c_device.h -- device-side building blocks shared by the CRC-32C kernels.
//
// Work decomposition:
//   * a *row* is 128 contiguous bytes of one block; an 8-lane *group* reads
//     one row with one 16-B load per lane (a 64-lane wave = 8 groups = 8 rows
//     of 8 different blocks per global_load_dwordx4 -> 8 full 128-B lines);
//   * lane li (0..7) of a group owns bytes [16li, 16li+16) of every row and
//     keeps one CRC register per 4-byte word of that slice ("braid" m = 0..3):
//     consecutive words of a braid are exactly 128 B apart, so each braid step
//     is  s = A^128(s ^ w)  -- the reference's slice-by-4 STEP4
//     (util/crc32c.cc:295-302) with tables for A^128 instead of A^4;
//   * the register kept per braid is the *pre-lookup* word c = s ^ w, so one
//     step is c' = T0[c.b0] ^ T1[c.b1] ^ T2[c.b2] ^ T3[c.b3] ^ w_next: four
//     v_perm (addresses), four ds_read_b32, two v_bitop3 (3-input xor);
//   * after the last row the 32 braid registers of a block are merged with
//     A^4 (in-lane, 3x), one lane-specific A^(116-16li) and a 3-step xor
//     reduction across the 8 lanes, using crc(X||Y) = A^|Y|(crc(X)) ^ crc(Y).
//
// LDS image (one workgroup per CU, 1024 threads):
//   [0, 128 KiB)   byte tables of A^128, replicated 32x so that lane l of every
//                  32-lane half-wave always reads bank (l & 31): conflict-free
//                  random lookups.  Byte address of entry (table t, index b):
//                      (t >> 1) << 16 | b << 8 | (t & 1) << 7 | (lane & 31) << 2
//                  so one and-or builds the address from the state word.
//   0x20000        nibble tables of A^4 (16 entries each: conflict-free)
//   0x20800        nibble tables of A^(116-16li), replicated per lane slot
//                  (lane & 31) like the byte tables: conflict-free.
//   kNibRowPow     nibble tables of A^(128 * 2^i), 9 <= i < 21 (ragged-path unit
//                  shifts of >= 512 rows); its first 9 slots: A^(2^i), i < 8,
//                  and A^-128 (the stream kernel's per-lane finish)
//   kNibNeg4       nibble tables of A^-4 (init injection)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_types.h"

namespace lsbm {

__device__ __forceinline__ uint32_t lds_load(const uint32_t* lds, uint32_t byte_addr) {
#ifdef LSBM_ABL_NO_LDS  // diagnostic builds only (tools/ablate.sh): a VALU op instead
  return byte_addr * 0x9e3779b1u;
#else
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
#endif
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 v_bitop3_b32
}

// The lane's part of a byte-table address, and each table's part (OR-ed into
// the v_perm constant L[t], whose bytes 0 and 2 land at bits 0..7 and
// 16..23 of the address, the state byte at bits 8..15).
#ifdef LSBM_LDS16
__device__ __forceinline__ uint32_t row_lane_base(uint32_t lane) { return (lane & 15u) << 2; }
constexpr uint32_t kRowTab[4] = {0x00u, 0x40u, 0x80u, 0xC0u};
#else
__device__ __forceinline__ uint32_t row_lane_base(uint32_t lane) { return (lane & 31u) << 2; }
constexpr uint32_t kRowTab[4] = {0x00u, 0x80u, 0x10000u, 0x10080u};
#endif

// One braid step: A^128(c) ^ w via the replicated byte tables (L[t] = the
// lane's constant part of the table-t address), i.e. the reference's STEP4
// (util/crc32c.cc:295-302) for a 128-byte stride, with the next word folded in.
__device__ __forceinline__ uint32_t row_step(const uint32_t* lds, uint32_t c, uint32_t w,
                                             uint32_t L0, uint32_t L1, uint32_t L2,
                                             uint32_t L3) {
  const uint32_t a0 = __builtin_amdgcn_perm(c, L0, 0x0c020400u);  // byte0 of c -> bits 8..15
  const uint32_t a1 = __builtin_amdgcn_perm(c, L1, 0x0c020500u);  // byte1
  const uint32_t a2 = __builtin_amdgcn_perm(c, L2, 0x0c020600u);  // byte2
  const uint32_t a3 = __builtin_amdgcn_perm(c, L3, 0x0c020700u);  // byte3
  return xor3(xor3(lds_load(lds, a0), lds_load(lds, a1), lds_load(lds, a2)), lds_load(lds, a3),
              w);
}

// M(v) for a matrix given as nibble tables in global memory (cached, rare use).
__device__ __forceinline__ uint32_t nib_glb(const uint32_t* __restrict__ tab, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) r ^= tab[q * 16 + ((v >> (4 * q)) & 15u)];
  return r;
}

// A^n(v) for any n >= 0 from the A^(2^k) tables.
__device__ __forceinline__ uint32_t advance_glb(const DevConsts* __restrict__ dc, uint32_t v,
                                                uint64_t n) {
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1u) v = nib_glb(dc->pow_nib[k], v);
  return v;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) {  // util/crc32c.h:31-34
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}
__device__ __forceinline__ uint32_t unmask_crc(uint32_t m) {  // util/crc32c.h:37-40
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}

// M(v) from uniform LDS nibble tables at `tab` (kNibA4, kNibA8, kNibA12:
// 512-B aligned, so the and-or merges the nibble field with the base).
template <uint32_t tab>
__device__ __forceinline__ uint32_t nib_uniform_lds(const uint32_t* lds, uint32_t v) {
  uint32_t t[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t f = q == 0 ? (v << 2) : (v >> (4 * q - 2));  // nibble q -> bits 2..5
    t[q] = lds_load(lds, ((f & 0x3cu) | tab) + q * 64);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// A^4(v): the uniform nibble tables, or (LSBM_LDS16) the lane's copy of the
// A^4 byte tables, as a row step with no next word.
__device__ __forceinline__ uint32_t adv4_lds(const uint32_t* lds, uint32_t v) {
#ifdef LSBM_LDS16
  const uint32_t lb = row_lane_base(threadIdx.x) | (kByteA4 >> 16) << 16;
  return row_step(lds, v, 0u, lb | kRowTab[0], lb | kRowTab[1], lb | kRowTab[2], lb | kRowTab[3]);
#else
  return nib_uniform_lds<kNibA4>(lds, v);
#endif
}

// The in-lane part of a merge: A^12(c0) ^ A^8(c1) ^ A^4(c2) ^ c3, the four
// braid words of a lane slice brought to its last word.  As a chain of three
// A^4 steps (three dependent LDS round trips), or (LSBM_MERGE_PAR) as three
// independent lookups in one round trip (the same VALU, the same loads).
__device__ __forceinline__ uint32_t lane_slice(const uint32_t* lds, uint32_t c0, uint32_t c1, uint32_t c2,
                                               uint32_t c3) {
#ifdef LSBM_MERGE_PAR
  return xor3(nib_uniform_lds<kNibA12>(lds, c0), nib_uniform_lds<kNibA8>(lds, c1),
              xor3(nib_uniform_lds<kNibA4>(lds, c2), c3, 0u));
#else
  uint32_t u = adv4_lds(lds, c0) ^ c1;
  u = adv4_lds(lds, u) ^ c2;
  return adv4_lds(lds, u) ^ c3;
#endif
}

// A^(116-16li)(v) from the lane-replicated LDS tables at kNibFin.
// lane_fin = kNibFin | (lane & 31) << 2.
__device__ __forceinline__ uint32_t fin_lds(const uint32_t* lds, uint32_t v, uint32_t lane_fin) {
  uint32_t t[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t f = q == 0 ? (v << 7) : (q == 1 ? (v << 3) : (v >> (4 * q - 7)));
    t[q] = lds_load(lds, ((f & 0x780u) | lane_fin) + q * 2048);  // nibble q -> bits 7..10
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// XOR of v over the 8 lanes of a group (DPP: swap neighbours, swap pairs,
// then mirror the two quads of each half-row); every lane gets the result.
__device__ __forceinline__ uint32_t group_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return v;
}

// Copy the prebuilt LDS image (DevConsts::lds_image) into LDS: every thread
// issues all of its 16-B loads before its first LDS write (one round trip).
template <uint32_t kThreads = kBlockThreads>
__device__ __forceinline__ void load_lds_tables(uint32_t* lds, const DevConsts* __restrict__ dc) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  constexpr uint32_t kChunks = kLdsBytes / 16;
  constexpr uint32_t kPer = (kChunks + kThreads - 1) / kThreads;
  const v4* __restrict__ src = reinterpret_cast<const v4*>(dc->lds_image);
  v4* dst = reinterpret_cast<v4*>(lds);
  v4 t[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < kChunks) t[k] = src[i];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < kChunks) dst[i] = t[k];
  }
  __syncthreads();
}

// Merge a group's 32 braid registers (c_m = pre-lookup word of braid m after
// the last row) into the raw CRC of the rows they cover, positioned at the
// end of the last row.  Every lane of the group gets the result.
__device__ __forceinline__ uint32_t merge_braids(const uint32_t* lds, uint32_t c0, uint32_t c1,
                                                 uint32_t c2, uint32_t c3, uint32_t lane_fin) {
  // in-lane: words at 16li + 0, 4, 8, 12 -> one register at 16li + 12
  uint32_t u = lane_slice(lds, c0, c1, c2, c3);
  // to the end of the row: A^(128 - (16li + 16)) then A^4 = A^(116 - 16li)
  u = fin_lds(lds, u, lane_fin);
  return group_xor(u);
}

// Two independent merges at once (the stream kernel's tail: the last saved
// block end and the segment's open block), their LDS lookups interleaved so
// that one round trip's latency covers both chains.
__device__ __forceinline__ void merge_braids2(const uint32_t* lds, uint32_t a0, uint32_t a1, uint32_t a2,
                                              uint32_t a3, uint32_t b0, uint32_t b1, uint32_t b2,
                                              uint32_t b3, uint32_t lane_fin, uint32_t& xa,
                                              uint32_t& xb) {
#ifdef LSBM_MERGE_PAR
  uint32_t u = lane_slice(lds, a0, a1, a2, a3), v = lane_slice(lds, b0, b1, b2, b3);
  u = fin_lds(lds, u, lane_fin);
  v = fin_lds(lds, v, lane_fin);
#else
  uint32_t u = adv4_lds(lds, a0), v = adv4_lds(lds, b0);
  u = adv4_lds(lds, u ^ a1);
  v = adv4_lds(lds, v ^ b1);
  u = adv4_lds(lds, u ^ a2);
  v = adv4_lds(lds, v ^ b2);
  u = fin_lds(lds, u ^ a3, lane_fin);
  v = fin_lds(lds, v ^ b3, lane_fin);
#endif
  xa = group_xor(u);
  xb = group_xor(v);
}

}  // namespace lsbm
