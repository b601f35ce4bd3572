// C++ host-side parity test of the batched block compression layer
// (include/lsbm/block_compression.h) against the per-block pattern of
// TableBuilder::WriteBlock (table/table_builder.cc:176-193) and ReadBlock
// (table/format.cc:104-145).  Expected compressed bytes come from the snappy
// oracle (oracle/snappy_oracle.c, pinned to libsnappy); the sealed output is
// then checked with the table layer.  Needs a GPU.
#include <stdio.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "lsbm/block_compression.h"
#include "lsbm/table_checksum.h"

extern "C" uint64_t so_compress(const uint8_t* in, uint32_t n, uint8_t* out);
extern "C" uint64_t so_max_compressed_length(uint64_t n);

static int fails = 0;
#define EXPECT(c)                                          \
  do {                                                     \
    if (!(c)) {                                            \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);   \
      fails++;                                             \
    }                                                      \
  } while (0)

static std::string make_block(std::mt19937_64& rng, size_t n, int kind) {
  std::string b(n, '\0');
  if (kind == 0) {  // db_bench-like: 50 printable bytes, repeated
    for (size_t i = 0; i < n; i++) b[i] = (i % 100) < 50 ? (char)(' ' + rng() % 95) : b[i - 50];
  } else if (kind == 1) {  // incompressible
    for (auto& c : b) c = (char)rng();
  } else if (kind == 2) {  // runs
    for (size_t i = 0; i < n; i++) b[i] = (char)('a' + (i / 37) % 3);
  } else {  // short-period text
    for (size_t i = 0; i < n; i++) b[i] = "leveldb-block-"[i % 14];
  }
  return b;
}

int main() {
  std::mt19937_64 rng(20261016);
  const size_t n = 1500;
  std::string raw;
  std::vector<uint64_t> off(1, 0);
  for (size_t i = 0; i < n; i++) {
    size_t len = rng() % 9000;
    if (i < 6) len = (size_t[]){0, 1, 15, 16, 4118, 100000}[i];
    raw += make_block(rng, len, (int)(rng() % 4));
    off.push_back(raw.size());
  }

  std::string contents;
  std::vector<uint64_t> coff;
  std::vector<uint8_t> types;
  lsbm::Status s = lsbm::CompressBlocks(0, raw.data(), off.data(), n, &contents, &coff, &types);
  EXPECT(s.ok());
  size_t n_snappy = 0;
  for (size_t i = 0; i < n && s.ok(); i++) {
    const uint64_t len = off[i + 1] - off[i];
    std::string c(so_max_compressed_length(len), '\0');
    c.resize(so_compress(reinterpret_cast<const uint8_t*>(raw.data() + off[i]), (uint32_t)len,
                         reinterpret_cast<uint8_t*>(&c[0])));
    const bool keep = c.size() < len - len / 8;  // table/table_builder.cc:187-188
    const std::string got = contents.substr(coff[i], coff[i + 1] - coff[i]);
    EXPECT(types[i] == (keep ? lsbm::kSnappyCompression : lsbm::kNoCompression));
    EXPECT(got == (keep ? c : raw.substr(off[i], len)));
    n_snappy += keep;
  }
  EXPECT(n_snappy > n / 4 && n_snappy < n);

  // ReadBlock: the contents decode back to the raw blocks
  std::string back;
  std::vector<uint64_t> boff;
  std::vector<uint8_t> ok;
  s = lsbm::UncompressBlocks(0, contents.data(), coff.data(), types.data(), n, &back, &boff, &ok);
  EXPECT(s.ok());
  EXPECT(back == raw);
  EXPECT(boff == off);

  // WriteRawBlock then ReadBlock's verify over the sealed image
  std::vector<uint64_t> sizes(n);
  for (size_t i = 0; i < n; i++) sizes[i] = coff[i + 1] - coff[i];
  uint64_t file_size = 0;
  std::vector<lsbm::BlockHandle> h = lsbm::LayoutBlocks(sizes, &file_size);
  std::string file(file_size, '\0');
  for (size_t i = 0; i < n; i++) memcpy(&file[h[i].offset], contents.data() + coff[i], sizes[i]);
  EXPECT(lsbm::SealBlocks(0, &file[0], file.size(), h.data(), types.data(), n).ok());
  for (size_t i = 0; i < n; i++) EXPECT((uint8_t)file[h[i].offset + sizes[i]] == types[i]);
  EXPECT(lsbm::VerifyBlocks(0, file.data(), file.size(), h.data(), n, nullptr).ok());

  // corruption: a snappy block cut by one byte, and later an unknown type
  size_t k = 0;
  while (types[k] != lsbm::kSnappyCompression) k++;
  std::string cut;
  std::vector<uint64_t> cutoff(1, 0);
  for (size_t i = 0; i < n; i++) {
    cut.append(contents, coff[i], coff[i + 1] - coff[i] - (i == k ? 1 : 0));
    cutoff.push_back(cut.size());
  }
  s = lsbm::UncompressBlocks(0, cut.data(), cutoff.data(), types.data(), n, &back, &boff, &ok);
  EXPECT(s.ToString() == "Corruption: corrupted compressed block contents");
  for (size_t i = 0; i < n; i++) EXPECT(ok[i] == (i == k ? 0 : 1));
  std::vector<uint8_t> bad = types;
  bad[k + 1] = 7;
  s = lsbm::UncompressBlocks(0, cut.data(), cutoff.data(), bad.data(), n, &back, &boff, &ok);
  EXPECT(s.ToString() == "Corruption: corrupted compressed block contents");  // block k comes first
  EXPECT(ok[k] == 0 && ok[k + 1] == 0);
  s = lsbm::UncompressBlocks(0, contents.data(), coff.data(), bad.data(), n, &back, &boff, &ok);
  EXPECT(s.ToString() == "Corruption: bad block type");

  // a block whose preamble claims 4 GiB among good ones: no 4 GiB window,
  // that block alone fails (it cannot expand 22x beyond its compressed size)
  {
    std::string mixed;
    std::vector<uint64_t> moff(1, 0);
    std::vector<uint8_t> mtypes;
    const size_t m = std::min<size_t>(n, 64), huge = m / 2;
    for (size_t i = 0; i < m; i++) {
      if (i == huge) {
        mixed += std::string("\xff\xff\xff\xff\x0f", 5) + std::string(40, 'a');
        mtypes.push_back(lsbm::kSnappyCompression);
      } else {
        mixed.append(contents, coff[i], coff[i + 1] - coff[i]);
        mtypes.push_back(types[i]);
      }
      moff.push_back(mixed.size());
    }
    s = lsbm::UncompressBlocks(0, mixed.data(), moff.data(), mtypes.data(), m, &back, &boff, &ok);
    EXPECT(s.ToString() == "Corruption: corrupted compressed block contents");
    for (size_t i = 0; i < m; i++) EXPECT(ok[i] == (i == huge ? 0 : 1));
    EXPECT(back.size() < (64u << 20));
    for (size_t i = 0; i < m; i++)
      if (i != huge) EXPECT(back.substr(boff[i], boff[i + 1] - boff[i]) == raw.substr(off[i], off[i + 1] - off[i]));
  }

  if (fails) {
    printf("FAILED %d\n", fails);
    return 1;
  }
  printf("OK %zu blocks, %zu snappy-compressed\n", n, n_snappy);
  return 0;
}
