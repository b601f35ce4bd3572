// ref_gpu_binding.cc -- TEST DRIVER for the Level-2 binding
// (integration/leveldb_gpu_checksum.h), built by oracle/Makefile `gpubind`
// from the reference's own table/ and util/ objects (build container) and run
// on the GPU box by tests/test_gpu_parity.py.
//
// A table image of 5,000 blocks laid out as TableBuilder writes them (block,
// then its 5-byte trailer: table/table_builder.cc:237-255) is sealed on the
// GPU through SealTrailersOnGpu; every trailer must be the one WriteRawBlock
// computes, and the reference's own ReadBlock (table/format.cc:66-148, with
// verify_checksums) must accept every block.  VerifyBlocksOnGpu must then pass
// the image and report "block checksum mismatch" for a flipped byte, as
// ReadBlock does on the same bytes.
//
// usage: ref_gpu_binding   (prints "OK ..." or FAIL lines; exit status)
#include <stdio.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "integration/leveldb_gpu_checksum.h"
#include "leveldb/env.h"
#include "leveldb/options.h"
#include "util/crc32c.h"

using namespace leveldb;

namespace {

int fails = 0;
#define EXPECT(c)                                         \
  do {                                                    \
    if (!(c)) {                                           \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);  \
      fails++;                                            \
    }                                                     \
  } while (0)

class StringFile : public RandomAccessFile {
 public:
  explicit StringFile(const std::string& s) : s_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result, char*) const {
    if (offset > s_.size()) return Status::IOError("read past end");
    *result = Slice(s_.data() + offset, std::min(n, (size_t)(s_.size() - offset)));
    return Status::OK();
  }

 private:
  const std::string& s_;
};

}  // namespace

int main() {
  std::mt19937_64 rng(20261017);
  const size_t n = 5000;
  std::vector<BlockHandle> h(n);
  std::vector<uint8_t> types(n);
  uint64_t off = 0;
  for (size_t i = 0; i < n; i++) {
    const uint64_t sz = i == 0 ? 0 : (i == 1 ? 4118 : rng() % 9000);
    h[i].set_offset(off);
    h[i].set_size(sz);
    types[i] = (i % 3 == 0) ? kSnappyCompression : kNoCompression;
    off += sz + kBlockTrailerSize;
  }
  std::string image(off, '\0');
  for (auto& c : image) c = (char)(' ' + rng() % 95);

  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  hipStream_t s;
  EXPECT(hipStreamCreate(&s) == hipSuccess);
  uint8_t* d_file = nullptr;
  EXPECT(hipMalloc(reinterpret_cast<void**>(&d_file), image.size()) == hipSuccess);
  EXPECT(hipMemcpy(d_file, image.data(), image.size(), hipMemcpyHostToDevice) == hipSuccess);

  // ---- seal: the trailers come back and are written into the host copy ----
  std::string sealed = image;
  Status st = SealTrailersOnGpu(d_file, image.size(), &sealed[0], h, types, s);
  EXPECT(st.ok());
  size_t read_ok = 0;
  StringFile file(sealed);
  ReadOptions ro;
  ro.verify_checksums = true;
  for (size_t i = 0; i < n; i++) {
    const char* block = sealed.data() + h[i].offset();
    char trailer[kBlockTrailerSize];
    trailer[0] = (char)types[i];
    const uint32_t crc = crc32c::Extend(crc32c::Value(block, h[i].size()), trailer, 1);
    EncodeFixed32(trailer + 1, crc32c::Mask(crc));  // table/table_builder.cc:245-249
    EXPECT(memcmp(trailer, block + h[i].size(), kBlockTrailerSize) == 0);
    if (types[i] == kNoCompression) {  // (no snappy here: ReadBlock would try to inflate)
      BlockContents bc;
      Status rs = ReadBlock(&file, ro, h[i], &bc);
      EXPECT(rs.ok());
      if (rs.ok()) {
        EXPECT(bc.data.size() == h[i].size() && memcmp(bc.data.data(), block, h[i].size()) == 0);
        if (bc.heap_allocated) delete[] bc.data.data();
        read_ok++;
      }
    }
  }

  // ---- verify: the sealed image passes; one flipped byte fails as ReadBlock fails ----
  EXPECT(hipMemcpy(d_file, sealed.data(), sealed.size(), hipMemcpyHostToDevice) == hipSuccess);
  std::vector<uint64_t> hh(2 * n);
  for (size_t i = 0; i < n; i++) {
    hh[2 * i] = h[i].offset();
    hh[2 * i + 1] = h[i].size();
  }
  uint64_t* d_h = nullptr;
  uint8_t* d_ok = nullptr;
  uint32_t* d_nbad = nullptr;
  EXPECT(hipMalloc(reinterpret_cast<void**>(&d_h), hh.size() * 8) == hipSuccess);
  EXPECT(hipMalloc(reinterpret_cast<void**>(&d_ok), n) == hipSuccess);
  EXPECT(hipMalloc(reinterpret_cast<void**>(&d_nbad), 4) == hipSuccess);
  EXPECT(hipMemcpy(d_h, hh.data(), hh.size() * 8, hipMemcpyHostToDevice) == hipSuccess);
  st = VerifyBlocksOnGpu(d_file, sealed.size(), d_h, n, d_ok, d_nbad, s);
  EXPECT(st.ok());
  const size_t bad = 2;  // a kNoCompression block
  sealed[h[bad].offset() + h[bad].size() / 2] ^= 0x10;
  EXPECT(hipMemcpy(d_file, sealed.data(), sealed.size(), hipMemcpyHostToDevice) == hipSuccess);
  st = VerifyBlocksOnGpu(d_file, sealed.size(), d_h, n, d_ok, d_nbad, s);
  BlockContents bc;
  const Status rs = ReadBlock(&file, ro, h[bad], &bc);
  EXPECT(st.IsCorruption() && rs.IsCorruption());
  EXPECT(st.ToString() == rs.ToString());
  std::vector<uint8_t> ok(n);
  EXPECT(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost) == hipSuccess);
  for (size_t i = 0; i < n; i++) EXPECT(ok[i] == (i == bad ? 0 : 1));
  // a handle whose trailer leaves the image, before the flipped block: ReadBlock's
  // "truncated block read" (table/format.cc:88-91) is the first failure
  const size_t cut = 1;
  hh[2 * cut + 1] = sealed.size() - h[cut].offset() - 3;
  EXPECT(hipMemcpy(d_h, hh.data(), hh.size() * 8, hipMemcpyHostToDevice) == hipSuccess);
  st = VerifyBlocksOnGpu(d_file, sealed.size(), d_h, n, d_ok, d_nbad, s);
  BlockHandle th;
  th.set_offset(hh[2 * cut]);
  th.set_size(hh[2 * cut + 1]);
  BlockContents tc;
  const Status ts = ReadBlock(&file, ro, th, &tc);
  EXPECT(st.IsCorruption() && ts.IsCorruption());
  EXPECT(st.ToString() == ts.ToString());
  EXPECT(st.ToString() == "Corruption: truncated block read");
  (void)hipFree(d_h);
  (void)hipFree(d_ok);
  (void)hipFree(d_nbad);
  (void)hipFree(d_file);
  (void)hipStreamDestroy(s);
  printf("%s (%zu blocks sealed, %zu read back through ReadBlock, verify: %s)\n", fails ? "FAILED" : "OK", n,
         read_ok, rs.ToString().c_str());
  return fails ? 1 : 0;
}
