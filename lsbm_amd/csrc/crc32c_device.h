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
//   * after the last row the 32 braid registers of a block are merged with
//     A^4 (in-lane) and A^16 / A^32 / A^64 (across the 8 lanes) into the raw
//     CRC, using the identity crc(X||Y) = A^|Y|(crc(X)) ^ crc(Y).
//
// LDS image (one workgroup per CU, 1024 threads):
//   [0, 128 KiB)   byte tables of A^128, replicated 32x so that lane l of every
//                  32-lane half-wave always reads bank (l & 31): conflict-free
//                  random lookups.  Byte address of entry (table t, index b):
//                      (t >> 1) << 16 | b << 8 | (t & 1) << 7 | (lane & 31) << 2
//                  so one and-or builds the address from the state word.
//   [128 KiB, +2K) nibble tables (16 entries each, hence conflict-free) of
//                  A^4, A^16, A^32, A^64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_types.h"

namespace lsbm {

__device__ __forceinline__ uint32_t lds_load(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// One braid step over the state word c = s ^ w: A^128(c) via the replicated
// byte tables (L[t] = the lane's constant part of the table-t address).
__device__ __forceinline__ uint32_t row_step(const uint32_t* lds, uint32_t c, uint32_t L0,
                                             uint32_t L1, uint32_t L2, uint32_t L3) {
  const uint32_t a0 = __builtin_amdgcn_perm(c, L0, 0x0c020400u);  // byte0 of c -> bits 8..15
  const uint32_t a1 = __builtin_amdgcn_perm(c, L1, 0x0c020500u);  // byte1
  const uint32_t a2 = __builtin_amdgcn_perm(c, L2, 0x0c020600u);  // byte2
  const uint32_t a3 = __builtin_amdgcn_perm(c, L3, 0x0c020700u);  // byte3
  return lds_load(lds, a0) ^ lds_load(lds, a1) ^ lds_load(lds, a2) ^ lds_load(lds, a3);
}

// M(v) for a matrix given as nibble tables in LDS at byte offset `tab`.
__device__ __forceinline__ uint32_t nib_lds(const uint32_t* lds, uint32_t tab, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) r ^= lds_load(lds, tab + q * 64 + ((v >> (4 * q)) & 15u) * 4);
  return r;
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

// Fill the LDS image from DevConsts (whole workgroup, ends with a barrier).
__device__ __forceinline__ void load_lds_tables(uint32_t* lds, const DevConsts* __restrict__ dc) {
  for (uint32_t w = threadIdx.x; w < kLdsByteTabBytes / 4; w += blockDim.x) {
    const uint32_t a = w << 2;
    const uint32_t t = ((a >> 16) << 1) | ((a >> 7) & 1u);
    const uint32_t b = (a >> 8) & 255u;
    lds[w] = dc->row_byte[t * 256 + b];
  }
  for (uint32_t w = threadIdx.x; w < 4 * 128; w += blockDim.x) {
    const uint32_t tab = w >> 7, e = w & 127u;
    const int k = tab == 0 ? 2 : (tab == 1 ? 4 : (tab == 2 ? 5 : 6));  // A^4, ^16, ^32, ^64
    lds[kLdsNibBase / 4 + w] = dc->pow_nib[k][e];
  }
  __syncthreads();
}

// Merge a group's 32 braid registers into the raw CRC of the rows they cover,
// positioned at the end of the last row.  li = lane within the 8-lane group.
// Valid on lane li == 7 only.
__device__ __forceinline__ uint32_t merge_braids(const uint32_t* lds, uint32_t s0, uint32_t s1,
                                                 uint32_t s2, uint32_t s3, uint32_t li) {
  // in-lane: words at 16li + 0, 4, 8, 12 -> one register at 16li + 12
  uint32_t u = nib_lds(lds, kNibA4, s0) ^ s1;
  u = nib_lds(lds, kNibA4, u) ^ s2;
  u = nib_lds(lds, kNibA4, u) ^ s3;
  // across lanes: pairs 16 B apart, then 32 B, then 64 B
  uint32_t t = __shfl_up(nib_lds(lds, kNibA16, u), 1, kGroupLanes);
  if (li & 1u) u ^= t;
  t = __shfl_up(nib_lds(lds, kNibA32, u), 2, kGroupLanes);
  if ((li & 3u) == 3u) u ^= t;
  t = __shfl_up(nib_lds(lds, kNibA64, u), 4, kGroupLanes);
  if (li == 7u) u ^= t;
  // lane 7 now holds the state positioned at the last word (row offset 124)
  return nib_lds(lds, kNibA4, u);
}

}  // namespace lsbm
