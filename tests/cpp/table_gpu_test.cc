// C++ host-side parity test of the batched SSTable trailer seal / verify
// (include/lsbm/table_checksum.h) against the per-block reference pattern of
// TableBuilder::WriteRawBlock (table/table_builder.cc:245-249) and ReadBlock
// (table/format.cc:95-103), computed with util/crc32c.h.  Needs a GPU.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <random>
#include <set>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "lsbm/log_checksum.h"
#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"
#include "util/crc32c.h"

static int fails = 0;
#define EXPECT(c)                                          \
  do {                                                     \
    if (!(c)) {                                            \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);   \
      fails++;                                             \
    }                                                      \
  } while (0)

static void encode_fixed32(char* p, uint32_t v) {
  for (int k = 0; k < 4; k++) p[k] = (char)(v >> (8 * k));
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);  // (a crash keeps what was printed)
  std::mt19937_64 rng(20261015);
  const size_t n = 3000;
  std::vector<uint64_t> sizes(n);
  for (auto& s : sizes) s = rng() % 9000;
  sizes[0] = 0;
  sizes[1] = 4118;  // a db_bench-sized data block
  uint64_t file_size = 0;
  std::vector<lsbm::BlockHandle> h = lsbm::LayoutBlocks(sizes, &file_size);
  std::string file(file_size, '\0');
  for (size_t i = 0; i < n; i++)
    for (uint64_t k = 0; k < sizes[i]; k++) file[h[i].offset + k] = (char)(' ' + rng() % 95);
  std::vector<uint8_t> types(n);
  for (auto& t : types) t = rng() & 1 ? lsbm::kSnappyCompression : lsbm::kNoCompression;

  lsbm::Status s = lsbm::SealBlocks(0, &file[0], file.size(), h.data(), types.data(), n);
  EXPECT(s.ok());
  // reference pattern, one block at a time
  for (size_t i = 0; i < n; i++) {
    const char* block = file.data() + h[i].offset;
    char trailer[5];
    trailer[0] = (char)types[i];
    uint32_t crc = leveldb::crc32c::Value(block, sizes[i]);
    crc = leveldb::crc32c::Extend(crc, trailer, 1);
    encode_fixed32(trailer + 1, leveldb::crc32c::Mask(crc));
    EXPECT(memcmp(trailer, block + sizes[i], 5) == 0);
    // ReadBlock's check on what was written
    const char* data = block;
    uint32_t stored;
    memcpy(&stored, data + sizes[i] + 1, 4);
    EXPECT(leveldb::crc32c::Unmask(stored) == leveldb::crc32c::Value(data, sizes[i] + 1));
  }
  std::vector<uint8_t> ok;
  s = lsbm::VerifyBlocks(0, file.data(), file.size(), h.data(), n, &ok);
  EXPECT(s.ok());
  // corrupt: a payload byte of block 7, the type byte of block 42, a crc byte of block 99
  file[h[7].offset + 3] ^= 0x40;
  file[h[42].offset + h[42].size] ^= 0x01;
  file[h[99].offset + h[99].size + 2] ^= 0x80;
  s = lsbm::VerifyBlocks(0, file.data(), file.size(), h.data(), n, &ok);
  EXPECT(s.IsCorruption());
  EXPECT(s.ToString() == "Corruption: block checksum mismatch");
  std::set<size_t> bad;
  for (size_t i = 0; i < n; i++)
    if (!ok[i]) bad.insert(i);
  EXPECT((bad == std::set<size_t>{7, 42, 99}));
  // a handle running past the end of the file
  lsbm::BlockHandle trunc{file_size - 3, 10};
  s = lsbm::VerifyBlocks(0, file.data(), file.size(), &trunc, 1, &ok);
  EXPECT(s.IsCorruption() && s.ToString() == "Corruption: truncated block read");

  // ---- SealTables / VerifyTables: many tables, one pipeline ----
  // 40 tables of 0..~6 MiB (some empty, one with its handles out of order,
  // one page-locked) sealed at once; every trailer checked against the
  // per-block reference pattern, then verify with one corrupted block.
  const size_t nt = 40;
  std::vector<std::string> files(nt);
  std::vector<std::vector<lsbm::BlockHandle>> hs(nt);
  std::vector<std::vector<uint8_t>> tys(nt);
  std::vector<lsbm::TableImage> im(nt);
  for (size_t t = 0; t < nt; t++) {
    const size_t nb = t == 3 ? 0 : (rng() % 1500);
    std::vector<uint64_t> sz(nb);
    for (auto& x : sz) x = rng() % 3 == 0 ? rng() % 200 : 3000 + rng() % 3000;
    uint64_t fs = 0;
    hs[t] = lsbm::LayoutBlocks(sz, &fs);
    files[t].assign(fs + 7, '\0');
    for (auto& c : files[t]) c = (char)(' ' + rng() % 95);
    tys[t].resize(nb);
    for (auto& y : tys[t]) y = rng() & 1;
    if (t == 5) std::reverse(hs[t].begin(), hs[t].end());  // handles out of offset order
    im[t] = lsbm::TableImage{&files[t][0], files[t].size(), hs[t].data(), tys[t].data(), nb};
  }
  // table 7 page-locked: its chunks are DMA-ed from the image itself
  const bool reg = hipHostRegister(&files[7][0], files[7].size(), hipHostRegisterDefault) == hipSuccess;
  EXPECT(reg);
  lsbm::Status st = lsbm::SealTables(0, im.data(), nt);
  EXPECT(st.ok());
  size_t checked = 0;
  for (size_t t = 0; t < nt; t++)
    for (size_t i = 0; i < hs[t].size(); i++, checked++) {
      const char* block = files[t].data() + hs[t][i].offset;
      char trailer[5];
      trailer[0] = (char)tys[t][i];
      uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(block, hs[t][i].size), trailer, 1);
      encode_fixed32(trailer + 1, leveldb::crc32c::Mask(crc));
      EXPECT(memcmp(trailer, block + hs[t][i].size, 5) == 0);
    }
  std::vector<uint8_t> oks;
  st = lsbm::VerifyTables(0, im.data(), nt, &oks);
  EXPECT(st.ok() && oks.size() == checked);
  files[9][hs[9][4].offset] ^= 0x08;  // a payload byte of table 9, block 4
  st = lsbm::VerifyTables(0, im.data(), nt, &oks);
  EXPECT(st.IsCorruption());
  size_t base9 = 0, nbad = 0;
  for (size_t t = 0; t < 9; t++) base9 += hs[t].size();
  for (size_t i = 0; i < oks.size(); i++) nbad += !oks[i];
  EXPECT(nbad == 1 && oks[base9 + 4] == 0);
  if (reg) (void)hipHostUnregister(&files[7][0]);

  fprintf(stderr, "section: small page-locked job\n");
  // ---- a small page-locked job (every image registered, <= 64 MiB): each
  // table one whole-image DMA and one kernel (or, LSBM_SMALL_LOCKED=zc, read
  // in place), tables spread over the stages: 6 tables, one empty, one with
  // its handles out of order, more tables than stages ----
  {
    const size_t st_n = 6;
    std::vector<std::string> f(st_n);
    std::vector<std::vector<lsbm::BlockHandle>> h(st_n);
    std::vector<std::vector<uint8_t>> y(st_n);
    std::vector<lsbm::TableImage> ti(st_n);
    std::vector<bool> regd(st_n, false);
    for (size_t t = 0; t < st_n; t++) {
      const size_t nb = t == 2 ? 0 : 200 + rng() % 1200;
      std::vector<uint64_t> sz(nb);
      for (auto& x : sz) x = rng() % 4 == 0 ? rng() % 100 : 3500 + rng() % 1200;
      uint64_t fs = 0;
      h[t] = lsbm::LayoutBlocks(sz, &fs);
      f[t].assign(fs + 3, '\0');
      for (auto& c : f[t]) c = (char)(' ' + rng() % 95);
      y[t].resize(nb);
      for (auto& x : y[t]) x = rng() % 3;
      if (t == 4) std::reverse(h[t].begin(), h[t].end());
      ti[t] = lsbm::TableImage{&f[t][0], f[t].size(), h[t].data(), y[t].data(), nb};
      regd[t] = hipHostRegister(&f[t][0], f[t].size(), hipHostRegisterDefault) == hipSuccess;
      EXPECT(regd[t]);
    }
    st = lsbm::SealTables(0, ti.data(), st_n);
    EXPECT(st.ok());
    size_t nblk = 0;
    for (size_t t = 0; t < st_n; t++)
      for (size_t i = 0; i < h[t].size(); i++, nblk++) {
        const char* block = f[t].data() + h[t][i].offset;
        char trailer[5];
        trailer[0] = (char)y[t][i];
        uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(block, h[t][i].size), trailer, 1);
        encode_fixed32(trailer + 1, leveldb::crc32c::Mask(crc));
        EXPECT(memcmp(trailer, block + h[t][i].size, 5) == 0);
      }
    std::vector<uint8_t> ok2;
    st = lsbm::VerifyTables(0, ti.data(), st_n, &ok2);
    EXPECT(st.ok() && ok2.size() == nblk && std::count(ok2.begin(), ok2.end(), 1) == (long)nblk);
    f[5][h[5][7].offset + h[5][7].size + 2] ^= 0x40;  // a stored crc byte of table 5, block 7
    st = lsbm::VerifyTables(0, ti.data(), st_n, &ok2);
    size_t base5 = 0;
    for (size_t t = 0; t < 5; t++) base5 += h[t].size();
    EXPECT(st.IsCorruption() && std::count(ok2.begin(), ok2.end(), 0) == 1 && ok2[base5 + 7] == 0);
    std::vector<uint8_t> ok1;  // one table per call, as TableBuilder::Finish
    st = lsbm::VerifyBlocks(0, f[1].data(), f[1].size(), h[1].data(), h[1].size(), &ok1);
    EXPECT(st.ok() && std::count(ok1.begin(), ok1.end(), 1) == (long)h[1].size());
    for (size_t t = 0; t < st_n; t++)
      if (regd[t]) (void)hipHostUnregister(&f[t][0]);

    // the sealed table read back through a read-only mapping of its file, as
    // the reference's PosixMmapReadableFile hands ReadBlock its bytes: the
    // layer may page-lock it for the call (read-only) or stage it; either
    // way every block verifies, and one flipped byte is found
    char path[] = "/tmp/lsbm_table_XXXXXX";
    const int fd = mkstemp(path);
    EXPECT(fd >= 0);
    if (fd >= 0) {
      f[1][h[1][3].offset + 1] ^= 0x01;  // block 3 of the file copy is corrupt
      EXPECT(write(fd, f[1].data(), f[1].size()) == (ssize_t)f[1].size());
      f[1][h[1][3].offset + 1] ^= 0x01;
      void* m = mmap(nullptr, f[1].size(), PROT_READ, MAP_PRIVATE, fd, 0);
      EXPECT(m != MAP_FAILED);
      if (m != MAP_FAILED) {
        for (int rep = 0; rep < 2; rep++) {  // (a second call: the lock was released)
          st = lsbm::VerifyBlocks(0, static_cast<const char*>(m), f[1].size(), h[1].data(), h[1].size(), &ok1);
          EXPECT(st.IsCorruption() && std::count(ok1.begin(), ok1.end(), 0) == 1 && ok1[3] == 0);
        }
        munmap(m, f[1].size());
      }
      close(fd);
      unlink(path);
    }

    // the same table from heap memory, as lsbm's ReadBlock holds it (pread
    // into new char[], table/format.cc:79-82): a writable char* image is
    // page-locked for the call and DMA-ed in place (one more per-call lock),
    // the same bytes as const char* are not (staged), and both verify
    const char* al = getenv("LSBM_AUTO_LOCK");
    const char* sl = getenv("LSBM_SMALL_LOCKED");
    const bool locks_on = !(al && atoi(al) == 0) && !(sl && strcmp(sl, "zc") == 0);
    const long l0 = lsbm_test_locks_taken();
    st = lsbm::VerifyBlocks(0, &f[1][0], f[1].size(), h[1].data(), h[1].size(), &ok1, lsbm::kImagesWritable);
    EXPECT(st.ok() && std::count(ok1.begin(), ok1.end(), 1) == (long)h[1].size());
    const long l1 = lsbm_test_locks_taken();
    EXPECT(l1 == l0 + (locks_on ? 1 : 0));
    st = lsbm::VerifyBlocks(0, static_cast<const char*>(&f[1][0]), f[1].size(), h[1].data(), h[1].size(), &ok1);
    EXPECT(st.ok() && lsbm_test_locks_taken() == l1);
    f[1][h[1][6].offset + 2] ^= 0x02;
    st = lsbm::VerifyBlocks(0, &f[1][0], f[1].size(), h[1].data(), h[1].size(), &ok1, lsbm::kImagesWritable);
    EXPECT(st.IsCorruption() && std::count(ok1.begin(), ok1.end(), 0) == 1 && ok1[6] == 0);
    f[1][h[1][6].offset + 2] ^= 0x02;
    EXPECT(lsbm_test_locked_ranges() == 0);
  }

  fprintf(stderr, "section: page locks next to the caller's registrations\n");
  // ---- per-call page locks next to the caller's own registrations: an image
  // that shares its first page with a range the caller registered, and one
  // that is registered in part.  The seal cannot lock them for the call, so it
  // stages them; trailers are still the reference's, and the caller's own
  // registrations are left as they were (unregistering them succeeds) ----
  {
    std::vector<uint64_t> sz(900);
    for (auto& x : sz) x = 3000 + rng() % 2000;
    uint64_t fs = 0;
    const std::vector<lsbm::BlockHandle> hh = lsbm::LayoutBlocks(sz, &fs);
    std::vector<uint8_t> yy(sz.size());
    for (auto& x : yy) x = rng() & 1;
    std::vector<char> big(2 * fs + (128u << 10));  // (img1 at +70017, img2 one image + 8 KiB later)
    for (auto& c : big) c = (char)(' ' + rng() % 95);
    char* base = big.data();
    char* mid = base + 70001;  // the caller's range ends inside a page ...
    char* img1 = mid + 16;     // ... that this image starts in
    EXPECT(hipHostRegister(base, (size_t)(mid - base), hipHostRegisterDefault) == hipSuccess);
    char* img2 = img1 + fs + 8192;  // registered in its first half by the caller
    EXPECT(hipHostRegister(img2, fs / 2, hipHostRegisterDefault) == hipSuccess);
    for (char* img : {img1, img2}) {
      fprintf(stderr, "seal %s\n", img == img1 ? "img1" : "img2");
      st = lsbm::SealBlocks(0, img, fs, hh.data(), yy.data(), hh.size());
      if (!st.ok()) printf("status: %s\n", st.ToString().c_str());
      EXPECT(st.ok());
      for (size_t i = 0; i < hh.size(); i++) {
        char trailer[5];
        trailer[0] = (char)yy[i];
        uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(img + hh[i].offset, hh[i].size), trailer, 1);
        encode_fixed32(trailer + 1, leveldb::crc32c::Mask(crc));
        EXPECT(memcmp(trailer, img + hh[i].offset + hh[i].size, 5) == 0);
      }
    }
    fprintf(stderr, "unregister\n");
    EXPECT(hipHostUnregister(img2) == hipSuccess);
    EXPECT(hipHostUnregister(base) == hipSuccess);
    fprintf(stderr, "section done\n");
  }

  // ---- error paths: a pipeline that fails with chunks in flight ----
  // (lsbm_test_fail_host_pipeline: the failure a copy or launch error would
  // give, after two chunks were enqueued).  The next call must neither collect
  // the failed call's chunks nor write their results: it seals byte for byte
  // what a clean run does, and verify / read report every record.
  {
    const size_t ft = 4;
    std::vector<std::string> f0(ft);
    std::vector<std::vector<lsbm::BlockHandle>> fh(ft);
    std::vector<std::vector<uint8_t>> fy(ft);
    for (size_t t = 0; t < ft; t++) {
      std::vector<uint64_t> sz(2800);
      for (auto& x : sz) x = 3000 + rng() % 3000;  // ~12 MiB per table: ~12 MiB chunks
      uint64_t fs = 0;
      fh[t] = lsbm::LayoutBlocks(sz, &fs);
      f0[t].assign(fs, '\0');
      for (auto& c : f0[t]) c = (char)(' ' + rng() % 95);
      fy[t].resize(sz.size());
      for (auto& y : fy[t]) y = rng() & 1;
    }
    auto images = [&](std::vector<std::string>& f) {
      std::vector<lsbm::TableImage> v(ft);
      for (size_t t = 0; t < ft; t++)
        v[t] = lsbm::TableImage{&f[t][0], f[t].size(), fh[t].data(), fy[t].data(), fh[t].size()};
      return v;
    };
    std::vector<std::string> fa = f0, fb = f0;
    std::vector<lsbm::TableImage> ia = images(fa), ib = images(fb);
    EXPECT(lsbm_test_fail_host_pipeline(2) == 0);
    st = lsbm::SealTables(0, ia.data(), ft);
    EXPECT(st.IsIOError() && st.ToString() == "IO error: injected fault");
    st = lsbm::SealTables(0, ib.data(), ft);
    EXPECT(st.ok());
    size_t nchk = 0;
    for (size_t t = 0; t < ft; t++) {
      // only the trailers differ from the unsealed image, and each is the reference's
      for (size_t i = 0; i < fh[t].size(); i++, nchk++) {
        const char* block = fb[t].data() + fh[t][i].offset;
        char trailer[5];
        trailer[0] = (char)fy[t][i];
        uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(block, fh[t][i].size), trailer, 1);
        encode_fixed32(trailer + 1, leveldb::crc32c::Mask(crc));
        EXPECT(memcmp(trailer, block + fh[t][i].size, 5) == 0);
        memcpy(&f0[t][fh[t][i].offset + fh[t][i].size], trailer, 5);
      }
      EXPECT(f0[t] == fb[t]);
    }
    EXPECT(lsbm_test_fail_host_pipeline(1) == 0);
    std::vector<uint8_t> okb;
    st = lsbm::VerifyTables(0, ib.data(), ft, &okb);
    EXPECT(st.IsIOError());
    st = lsbm::VerifyTables(0, ib.data(), ft, &okb);
    EXPECT(st.ok() && okb.size() == nchk);
    for (uint8_t o : okb) EXPECT(o == 1);

    // the log layer (log_checksum.cc): ~40 MiB of records, ~10 MiB chunks
    lsbm::log::BatchWriter w;
    std::vector<std::string> recs;
    size_t total = 0;
    while (total < (40u << 20)) {
      std::string r(rng() % 5000, '\0');
      for (auto& c : r) c = (char)(' ' + rng() % 95);
      total += r.size();
      w.AddRecord(r.data(), r.size());
      recs.push_back(std::move(r));
    }
    EXPECT(lsbm_test_fail_host_pipeline(2) == 0);
    st = w.Seal(0);
    EXPECT(st.IsIOError());
    st = w.Seal(0);  // the same headers again, from scratch
    EXPECT(st.ok());
    const std::string& img = w.contents();
    size_t bad_headers = 0;
    for (uint64_t hd : w.headers()) {
      const uint8_t* hp = reinterpret_cast<const uint8_t*>(img.data() + hd);
      const size_t len = hp[4] | (hp[5] << 8);
      uint32_t stored;
      memcpy(&stored, hp, 4);
      bad_headers += leveldb::crc32c::Unmask(stored) != leveldb::crc32c::Value(img.data() + hd + 6, len + 1);
    }
    EXPECT(bad_headers == 0);
    struct CountingReporter : lsbm::log::Reporter {
      size_t n = 0;
      void Corruption(size_t, const lsbm::Status&) override { n++; }
    } rep;
    std::vector<std::string> got;
    std::vector<uint64_t> offs;
    EXPECT(lsbm_test_fail_host_pipeline(1) == 0);
    st = lsbm::log::ReadLog(0, img.data(), img.size(), &rep, &got, &offs);
    EXPECT(st.IsIOError());
    st = lsbm::log::ReadLog(0, img.data(), img.size(), &rep, &got, &offs);
    EXPECT(st.ok() && rep.n == 0 && got == recs);
    EXPECT(lsbm_test_fail_host_pipeline(-1) == 0);
  }
  printf("%s (%zu blocks, %llu bytes; %zu blocks over %zu tables)\n", fails ? "FAILED" : "OK", n,
         (unsigned long long)file_size, checked, nt);
  return fails ? 1 : 0;
}
