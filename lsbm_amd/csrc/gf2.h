// gf2.h -- CRC-32C as linear algebra over GF(2) (host side, used to build every
// device table; nothing here is copied from the reference's literal tables).
//
// The reference advances its CRC register one byte at a time with
//     l = table0_[(l ^ b) & 0xff] ^ (l >> 8)            (util/crc32c.cc:291-294)
// which, with b = 0, is a linear map A on 32-bit states ("advance one zero
// byte").  Every kernel in this library is built from powers of A:
//   * the slice-by-4 step over a 4-byte little-endian word w is A^4(l ^ w)
//     (util/crc32c.cc:295-302); a step that also skips S-4 bytes is A^S(l ^ w);
//   * crc(X || Y) = A^|Y|(crc_raw(X)) ^ crc_raw(Y) for the raw (no inversion)
//     CRC, which is what lets lanes, braids and segments be combined;
//   * A is invertible (the polynomial has a non-zero constant term), so
//     trailing zero padding can be removed with A^-z.
// A 32x32 GF(2) matrix is stored as its 32 columns: M(v) = XOR_{bit b of v} col[b].
#pragma once
#include <stdint.h>
#include <string.h>

namespace lsbm {
namespace gf2 {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli (util/crc32c.cc:5-6)

struct Mat {
  uint32_t col[32];
};

inline uint32_t apply(const Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int b = 0; b < 32; b++)
    if (v >> b & 1u) r ^= m.col[b];
  return r;
}

inline Mat mul(const Mat& a, const Mat& b) {  // (a*b)(v) = a(b(v))
  Mat r;
  for (int k = 0; k < 32; k++) r.col[k] = apply(a, b.col[k]);
  return r;
}

inline Mat identity() {
  Mat r;
  for (int k = 0; k < 32; k++) r.col[k] = 1u << k;
  return r;
}

// One zero *bit* through the reflected register, and its inverse.
inline uint32_t bit_step(uint32_t l) { return (l >> 1) ^ (kPoly & (0u - (l & 1u))); }
inline uint32_t bit_unstep(uint32_t y) {
  // kPoly has bit 31 set, so y's top bit tells whether the poly was folded in.
  return (y >> 31) ? (((y ^ kPoly) << 1) | 1u) : (y << 1);
}

inline Mat from_fn(uint32_t (*f)(uint32_t)) {
  Mat r;
  for (int k = 0; k < 32; k++) r.col[k] = f(1u << k);
  return r;
}

// A^e for e >= 0 (advance e zero bytes) or e < 0 (retreat |e| bytes).
inline Mat byte_pow(int64_t e) {
  Mat base = from_fn(e >= 0 ? bit_step : bit_unstep);
  uint64_t bits = (uint64_t)(e >= 0 ? e : -e) * 8u;  // bytes -> bit steps
  Mat r = identity();
  while (bits) {
    if (bits & 1u) r = mul(base, r);
    base = mul(base, base);
    bits >>= 1;
  }
  return r;
}

// Byte tables: tab[p*256 + b] = M(b << 8p), p = 0..3.  For M = A^S these are
// the S-byte generalisation of the reference's slice-by-4 tables:
// A^4 gives table3_, table2_, table1_, table0_ for p = 0, 1, 2, 3.
inline void byte_tables(const Mat& m, uint32_t* tab1024) {
  for (int p = 0; p < 4; p++)
    for (uint32_t b = 0; b < 256; b++) tab1024[p * 256 + b] = apply(m, b << (8 * p));
}

// Nibble tables: tab[q*16 + v] = M(v << 4q), q = 0..7.  16 entries per table:
// every table sits in 16 distinct LDS banks, so random lookups never conflict.
inline void nibble_tables(const Mat& m, uint32_t* tab128) {
  for (int q = 0; q < 8; q++)
    for (uint32_t v = 0; v < 16; v++) tab128[q * 16 + v] = apply(m, v << (4 * q));
}

}  // namespace gf2
}  // namespace lsbm
