// crc32c_host.cc -- the scalar CRC-32C behind include/util/crc32c.h.
//
// Exports the reference's one out-of-line symbol, leveldb::crc32c::Extend
// (util/crc32c.h:17, defined at util/crc32c.cc:286-329), so table/ and
// common/log_* link unchanged, plus the C names lsbm_crc32c_{extend,value,
// mask,unmask}.  This is the reference's *scalar* API (single small records,
// WAL headers, the 1-byte type extension); batches of blocks use the GPU
// entry points in crc32c_engine.hip, which never fall back to this code.
//
// Same function as the reference (CRC-32C, reflected 0x82F63B78, pre/post
// inversion, alignment-independent) but not the same algorithm: on x86 hosts
// with SSE4.2 it uses the crc32 instruction (3 interleaved streams merged with
// GF(2) shifts); elsewhere a slice-by-8 table walk with generated tables.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <mutex>

#include "../../include/lsbm_crc32c.h"
#include "../../include/util/crc32c.h"
#include "gf2.h"

namespace lsbm {
namespace {

struct HostTables {
  uint32_t slice8[8][256];  // slice8[k][b] = A^(k+1)(b)
  uint32_t shift_1k[4][256];  // byte tables of A^1024 (merging hw streams)
  uint32_t shift_2k[4][256];  // byte tables of A^2048
  bool have_sse42 = false;
};

HostTables* g_tabs = nullptr;
std::once_flag g_tabs_once;

void build_host_tables() {
  HostTables* t = new HostTables();
  for (int k = 0; k < 8; k++) {
    gf2::Mat m = gf2::byte_pow(k + 1);
    for (uint32_t b = 0; b < 256; b++) t->slice8[k][b] = gf2::apply(m, b);
  }
  gf2::byte_tables(gf2::byte_pow(1024), &t->shift_1k[0][0]);
  gf2::byte_tables(gf2::byte_pow(2048), &t->shift_2k[0][0]);
#if defined(__x86_64__)
  __builtin_cpu_init();
  t->have_sse42 = __builtin_cpu_supports("sse4.2");
#endif
  g_tabs = t;
}

inline const HostTables& tabs() {
  std::call_once(g_tabs_once, build_host_tables);
  return *g_tabs;
}

inline uint32_t shift_by(const uint32_t (*tb)[256], uint32_t v) {
  return tb[0][v & 0xff] ^ tb[1][(v >> 8) & 0xff] ^ tb[2][(v >> 16) & 0xff] ^ tb[3][v >> 24];
}

// Portable raw update: state l (already inverted) over p[0, n).
uint32_t raw_portable(const HostTables& t, uint32_t l, const uint8_t* p, size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    l = t.slice8[0][(l ^ *p++) & 0xff] ^ (l >> 8);
    n--;
  }
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    w ^= l;
    l = t.slice8[7][w & 0xff] ^ t.slice8[6][(w >> 8) & 0xff] ^ t.slice8[5][(w >> 16) & 0xff] ^
        t.slice8[4][(w >> 24) & 0xff] ^ t.slice8[3][(w >> 32) & 0xff] ^
        t.slice8[2][(w >> 40) & 0xff] ^ t.slice8[1][(w >> 48) & 0xff] ^ t.slice8[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) l = t.slice8[0][(l ^ *p++) & 0xff] ^ (l >> 8);
  return l;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t raw_sse42(const HostTables& t, uint32_t l,
                                                     const uint8_t* p, size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    l = __builtin_ia32_crc32qi(l, *p++);
    n--;
  }
  // Three independent 1 KiB streams hide the crc32 instruction's latency;
  // a || b || c = A^2048(a) ^ A^1024(b) ^ c on the raw register.
  while (n >= 3072) {
    uint64_t a = l, b = 0, c = 0;
    for (int k = 0; k < 1024; k += 8) {
      uint64_t wa, wb, wc;
      memcpy(&wa, p + k, 8);
      memcpy(&wb, p + 1024 + k, 8);
      memcpy(&wc, p + 2048 + k, 8);
      a = __builtin_ia32_crc32di(a, wa);
      b = __builtin_ia32_crc32di(b, wb);
      c = __builtin_ia32_crc32di(c, wc);
    }
    l = shift_by(t.shift_2k, (uint32_t)a) ^ shift_by(t.shift_1k, (uint32_t)b) ^ (uint32_t)c;
    p += 3072;
    n -= 3072;
  }
  uint64_t l64 = l;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    l64 = __builtin_ia32_crc32di(l64, w);
    p += 8;
    n -= 8;
  }
  l = (uint32_t)l64;
  while (n--) l = __builtin_ia32_crc32qi(l, *p++);
  return l;
}
#endif

}  // namespace

uint32_t host_extend(uint32_t crc, const uint8_t* p, size_t n) {
  const HostTables& t = tabs();
  uint32_t l = crc ^ 0xffffffffu;
#if defined(__x86_64__)
  if (t.have_sse42) return raw_sse42(t, l, p, n) ^ 0xffffffffu;
#endif
  return raw_portable(t, l, p, n) ^ 0xffffffffu;
}

}  // namespace lsbm

namespace leveldb {
namespace crc32c {
__attribute__((visibility("default"))) uint32_t Extend(uint32_t init_crc, const char* data,
                                                       size_t n) {
  return lsbm::host_extend(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}
}  // namespace crc32c
}  // namespace leveldb

extern "C" {
__attribute__((visibility("default"))) uint32_t lsbm_crc32c_extend(uint32_t init_crc,
                                                                   const char* data, size_t n) {
  if (n == 0) return init_crc;
  if (!data) return init_crc;
  return lsbm::host_extend(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}
__attribute__((visibility("default"))) uint32_t lsbm_crc32c_value(const char* data, size_t n) {
  return lsbm_crc32c_extend(0, data, n);
}
__attribute__((visibility("default"))) uint32_t lsbm_crc32c_mask(uint32_t crc) {
  return leveldb::crc32c::Mask(crc);
}
__attribute__((visibility("default"))) uint32_t lsbm_crc32c_unmask(uint32_t m) {
  return leveldb::crc32c::Unmask(m);
}
}
