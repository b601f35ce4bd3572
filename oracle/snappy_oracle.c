/* snappy_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU parity checker for the
 * GPU snappy block codec (lsbm_amd/csrc/snappy_kernels.hip).  Never linked into
 * the product; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it.
 *
 * The reference compresses SSTable blocks with the third-party libsnappy,
 * through port::Snappy_Compress / Snappy_GetUncompressedLength /
 * Snappy_Uncompress (port/port_posix.h:119-150 -> snappy::RawCompress,
 * snappy::GetUncompressedLength, snappy::RawUncompress), called from
 * TableBuilder::WriteBlock (table/table_builder.cc:181-193) and ReadBlock
 * (table/format.cc:124-141).  libsnappy is not vendored in /root/reference and
 * is not installed here; this file restates its published raw format
 * (format_description.txt: varint32 length, then literal / copy-1 / copy-2 /
 * copy-4 tags) and its compressor (snappy.cc CompressFragment: 64 KiB
 * fragments, a uint16 hash table of min(2^15, pow2 >= fragment) entries
 * (>= 256), HashBytes = ((x * 0x1e35a7bd) >> (32 - 15)) & mask, the 32-probe
 * skip heuristic, matches re-probed at ip-1 / ip, copies of at most 64 bytes
 * (a 68+ tail split as 60 + rest), 1-byte-offset copies for len < 12 and
 * offset < 2048).  Parity is pinned against the libsnappy that ships inside
 * the image's pyarrow 25.0.0 (pyarrow.Codec("snappy") is snappy::RawCompress /
 * RawUncompress): tests/golden/make_snappy_fixture.py records its outputs and
 * tests/test_snappy.py checks this restatement byte-for-byte against them.
 * The 2^15-entry table and the masked top-15-bit hash are the libsnappy >= 1.1.10
 * compressor; the 2^14 table or the top-log2(size)-bit hash of older releases
 * disagree with that library on a third of the pinning inputs, so the reference
 * linked against an older libsnappy would write different (equally valid)
 * compressed blocks.  Decompression is version-independent.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define SO_BLOCK_LOG 16
#define SO_BLOCK_SIZE (1u << SO_BLOCK_LOG)
#define SO_MAX_TABLE_BITS 15
#define SO_MAX_TABLE (1u << SO_MAX_TABLE_BITS)
#define SO_MIN_TABLE 256u
#define SO_INPUT_MARGIN 15

static uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* snappy::MaxCompressedLength */
uint64_t so_max_compressed_length(uint64_t n) { return 32 + n + n / 6; }

/* snappy::GetUncompressedLength: varint32, at most 5 bytes, the 5th < 16.
 * Returns the number of preamble bytes (>= 1) or 0 on failure. */
int so_get_uncompressed_length(const uint8_t* in, uint64_t n, uint32_t* out) {
  uint32_t v = 0;
  for (int i = 0; i < 5; i++) {
    if ((uint64_t)i >= n) return 0;
    const uint32_t b = in[i];
    if (i == 4 && b >= 16) return 0;
    v |= (b & 127u) << (7 * i);
    if (b < 128) {
      *out = v;
      return i + 1;
    }
  }
  return 0;
}

/* snappy::RawUncompress into out[0, cap).  Succeeds iff the tags consume the
 * input exactly, every literal lies inside the input, every copy has
 * 1 <= offset <= bytes produced so far, the output never exceeds the preamble
 * length, and ends exactly at it.  Returns 1 / 0; *produced = ulength. */
int so_uncompress(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* produced) {
  uint32_t ulen;
  const int pre = so_get_uncompressed_length(in, n, &ulen);
  if (!pre) return 0;
  if (ulen > cap) return 0;
  uint64_t ip = (uint64_t)pre, op = 0;
  while (ip < n) {
    const uint32_t c = in[ip++];
    const uint32_t kind = c & 3u;
    if (kind == 0) {
      uint64_t len = (c >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60; /* 1..4 extra length bytes */
        if (ip + nb > n) return 0;
        uint64_t v = 0;
        for (uint32_t i = 0; i < nb; i++) v |= (uint64_t)in[ip + i] << (8 * i);
        ip += nb;
        len = v + 1;
      }
      if (len > n - ip) return 0;
      if (len > ulen - op) return 0;
      memcpy(out + op, in + ip, len);
      ip += len;
      op += len;
    } else {
      uint64_t len, off;
      if (kind == 1) {
        if (ip + 1 > n) return 0;
        len = 4 + ((c >> 2) & 7u);
        off = ((uint64_t)(c >> 5) << 8) | in[ip];
        ip += 1;
      } else if (kind == 2) {
        if (ip + 2 > n) return 0;
        len = (c >> 2) + 1;
        off = (uint64_t)in[ip] | ((uint64_t)in[ip + 1] << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) return 0;
        len = (c >> 2) + 1;
        off = ld32(in + ip);
        ip += 4;
      }
      if (off == 0 || off > op) return 0;
      if (len > ulen - op) return 0;
      for (uint64_t i = 0; i < len; i++) out[op + i] = out[op - off + i];
      op += len;
    }
  }
  if (op != ulen) return 0;
  *produced = op;
  return 1;
}

static uint32_t table_size_for(uint32_t n) {
  if (n > SO_MAX_TABLE) return SO_MAX_TABLE;
  if (n < SO_MIN_TABLE) return SO_MIN_TABLE;
  uint32_t t = SO_MIN_TABLE;
  while (t < n) t <<= 1;
  return t;
}

static uint32_t hash_bytes(uint32_t bytes, uint32_t mask) {
  return ((bytes * 0x1e35a7bdu) >> (32 - SO_MAX_TABLE_BITS)) & mask;
}

static uint8_t* emit_literal(uint8_t* op, const uint8_t* lit, uint32_t len) {
  const uint32_t n = len - 1;
  if (n < 60) {
    *op++ = (uint8_t)(n << 2);
  } else {
    uint32_t count = 0;
    for (uint32_t t = n; t; t >>= 8) count++;
    *op++ = (uint8_t)((59 + count) << 2);
    for (uint32_t i = 0; i < count; i++) *op++ = (uint8_t)(n >> (8 * i));
  }
  memcpy(op, lit, len);
  return op + len;
}

static uint8_t* emit_copy_le64(uint8_t* op, uint32_t off, uint32_t len, int lt12) {
  if (lt12 && off < 2048) {
    *op++ = (uint8_t)(1u + ((len - 4) << 2) + ((off >> 3) & 0xe0u));
    *op++ = (uint8_t)off;
  } else {
    *op++ = (uint8_t)(2u + ((len - 1) << 2));
    *op++ = (uint8_t)off;
    *op++ = (uint8_t)(off >> 8);
  }
  return op;
}

static uint8_t* emit_copy(uint8_t* op, uint32_t off, uint32_t len) {
  if (len < 12) return emit_copy_le64(op, off, len, 1);
  while (len >= 68) {
    op = emit_copy_le64(op, off, 64, 0);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_le64(op, off, 60, 0);
    len -= 60;
  }
  return emit_copy_le64(op, off, len, len < 12);
}

static uint32_t match_len(const uint8_t* s1, const uint8_t* s2, const uint8_t* s2_end) {
  uint32_t m = 0;
  while (s2 + m < s2_end && s1[m] == s2[m]) m++;
  return m;
}

/* snappy.cc CompressFragment over one fragment (<= 64 KiB). */
static uint8_t* compress_fragment(const uint8_t* in, uint32_t n, uint8_t* op, uint16_t* table,
                                  uint32_t tsize) {
  const uint32_t mask = tsize - 1;
  const uint8_t* ip = in;
  const uint8_t* const end = in + n;
  const uint8_t* next_emit = ip;
  memset(table, 0, tsize * sizeof(uint16_t));
  if (n >= SO_INPUT_MARGIN) {
    const uint8_t* const limit = in + n - SO_INPUT_MARGIN;
    for (;;) {
      next_emit = ip++;
      uint32_t skip = 32;
      const uint8_t* cand;
      for (;;) {
        const uint32_t data = ld32(ip);
        const uint32_t h = hash_bytes(data, mask);
        const uint32_t step = skip >> 5;
        skip += step;
        const uint8_t* next_ip = ip + step;
        if (next_ip > limit) {
          ip = next_emit;
          goto remainder;
        }
        cand = in + table[h];
        table[h] = (uint16_t)(ip - in);
        if (ld32(cand) == data) break;
        ip = next_ip;
      }
      op = emit_literal(op, next_emit, (uint32_t)(ip - next_emit));
      for (;;) {
        const uint8_t* base = ip;
        const uint32_t matched = 4 + match_len(cand + 4, ip + 4, end);
        ip += matched;
        op = emit_copy(op, (uint32_t)(base - cand), matched);
        next_emit = ip;
        if (ip >= limit) goto remainder;
        table[hash_bytes(ld32(ip - 1), mask)] = (uint16_t)(ip - in - 1);
        const uint32_t data = ld32(ip);
        const uint32_t h = hash_bytes(data, mask);
        cand = in + table[h];
        table[h] = (uint16_t)(ip - in);
        if (ld32(cand) != data) break;
      }
    }
  }
remainder:
  if (next_emit < end) op = emit_literal(op, next_emit, (uint32_t)(end - next_emit));
  return op;
}

/* snappy::RawCompress: varint32 length, then 64 KiB fragments compressed
 * independently.  out needs so_max_compressed_length(n) bytes.  Returns the
 * compressed size. */
uint64_t so_compress(const uint8_t* in, uint32_t n, uint8_t* out) {
  uint16_t table[SO_MAX_TABLE];
  uint8_t* op = out;
  uint32_t v = n;
  while (v >= 128) {
    *op++ = (uint8_t)(v | 128);
    v >>= 7;
  }
  *op++ = (uint8_t)v;
  for (uint32_t pos = 0; pos < n;) {
    const uint32_t frag = n - pos < SO_BLOCK_SIZE ? n - pos : SO_BLOCK_SIZE;
    op = compress_fragment(in + pos, frag, op, table, table_size_for(frag));
    pos += frag;
  }
  return (uint64_t)(op - out);
}

/* Batch driver (CPU baseline): compress block i = in[off[i], off[i+1]) into
 * out + oo[i] (oo[i] = sum of max lengths before i); sizes to osz[i]. */
void so_compress_batch(const uint8_t* in, const uint64_t* off, uint64_t n, uint8_t* out,
                       const uint64_t* oo, uint64_t* osz) {
  for (uint64_t i = 0; i < n; i++)
    osz[i] = so_compress(in + off[i], (uint32_t)(off[i + 1] - off[i]), out + oo[i]);
}

/* Batch driver: uncompress block i = in[off[i], off[i+1]) into out + uo[i]
 * (capacity uo[i+1] - uo[i]); ok[i] = success.  Returns the failures. */
uint64_t so_uncompress_batch(const uint8_t* in, const uint64_t* off, uint64_t n, uint8_t* out,
                             const uint64_t* uo, uint8_t* ok) {
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t got = 0;
    ok[i] = (uint8_t)so_uncompress(in + off[i], off[i + 1] - off[i], out + uo[i],
                                   uo[i + 1] - uo[i], &got);
    bad += !ok[i];
  }
  return bad;
}
