// Concurrent callers of the table layer on one device (include/lsbm/
// table_checksum.h), as the reference's compaction, writer and reader threads
// would make them (util/env_posix.cc:546-586): C threads each seal their own
// 16 MiB table (one table per call, TableBuilder::Finish's granularity,
// lsbm/db_impl.cc:843-892), then verify it.
//
// Checks: the trailers are byte-identical to the same calls made one after
// another, and to WriteRawBlock's pattern computed with util/crc32c.h
// (table/table_builder.cc:245-249); every block verifies; and the concurrent
// calls take measurably less wall time than the serial ones (each caller
// leases its own session: stages, streams and pinned staging).
//
//   concurrent_seal_test [callers=4] [reps=8] [pinned=0] [zero_copy_max_mb=64]
// prints "OK serial_ms=... concurrent_ms=... speedup=..." or FAIL lines.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"
#include "util/crc32c.h"

static int fails = 0;
#define EXPECT(c)                                        \
  do {                                                   \
    if (!(c)) {                                          \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      fails++;                                           \
    }                                                    \
  } while (0)

namespace {
double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Table {
  std::vector<char> img;
  std::vector<lsbm::BlockHandle> h;
  std::vector<uint8_t> types;
};

void make_table(Table* t, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<uint64_t> sizes((16u << 20) / 4123);
  for (auto& s : sizes) s = 3900 + rng() % 400;  // db_bench-like data blocks
  uint64_t fs = 0;
  t->h = lsbm::LayoutBlocks(sizes, &fs);
  t->img.assign(fs, 0);
  for (size_t i = 0; i + 8 <= fs; i += 8) {
    uint64_t r = rng();
    for (int k = 0; k < 8; k++, r >>= 8) t->img[i + k] = (char)(' ' + (r & 0xff) % 95);
  }
  t->types.resize(sizes.size());
  for (auto& x : t->types) x = rng() & 1;
}

bool reference_trailers_ok(const Table& t) {
  for (size_t i = 0; i < t.h.size(); i++) {
    const char* b = t.img.data() + t.h[i].offset;
    uint32_t crc = leveldb::crc32c::Value(b, t.h[i].size);
    const char type = (char)t.types[i];
    crc = leveldb::crc32c::Extend(crc, &type, 1);
    const uint32_t m = leveldb::crc32c::Mask(crc);
    char want[5] = {type, (char)m, (char)(m >> 8), (char)(m >> 16), (char)(m >> 24)};
    if (memcmp(want, b + t.h[i].size, 5) != 0) return false;
  }
  return true;
}

lsbm::Status seal(Table& t) {
  return lsbm::SealBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.types.data(), t.h.size());
}
}  // namespace

int main(int argc, char** argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  const bool pinned = argc > 3 && atoi(argv[3]) != 0;
  // page-locked one-table jobs: read in place by the kernel (the default) or,
  // with 0, DMA-ed in chunks through the session's copy stream
  if (argc > 4) lsbm_test_zero_copy_max_mb(atoi(argv[4]));
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  std::vector<Table> ts(callers);
  for (int c = 0; c < callers; c++) make_table(&ts[c], 1000 + c);
  if (pinned)
    for (auto& t : ts) EXPECT(hipHostRegister(t.img.data(), t.img.size(), hipHostRegisterDefault) == hipSuccess);
  // serial reference images (and warm sessions / pool)
  std::vector<std::vector<char>> serial_img(callers);
  for (int c = 0; c < callers; c++) {
    EXPECT(seal(ts[c]).ok());
    EXPECT(reference_trailers_ok(ts[c]));
    serial_img[c] = ts[c].img;
  }
  {  // every caller's session exists before timing
    std::vector<std::thread> th;
    for (int c = 0; c < callers; c++) th.emplace_back([&, c] { EXPECT(seal(ts[c]).ok()); });
    for (auto& x : th) x.join();
  }
  double best_serial = 1e9, best_conc = 1e9;
  for (int round = 0; round < 3; round++) {
    // scrub the trailers, so that every round writes them again
    for (auto& t : ts)
      for (auto& hd : t.h) memset(t.img.data() + hd.offset + hd.size, 0, 5);
    double t0 = now();
    for (int r = 0; r < reps; r++)
      for (int c = 0; c < callers; c++) EXPECT(seal(ts[c]).ok());
    best_serial = std::min(best_serial, now() - t0);
    for (int c = 0; c < callers; c++) EXPECT(ts[c].img == serial_img[c]);
    for (auto& t : ts)
      for (auto& hd : t.h) memset(t.img.data() + hd.offset + hd.size, 0, 5);
    std::atomic<int> bad{0};
    t0 = now();
    std::vector<std::thread> th;
    for (int c = 0; c < callers; c++)
      th.emplace_back([&, c] {
        for (int r = 0; r < reps; r++)
          if (!seal(ts[c]).ok()) bad++;
      });
    for (auto& x : th) x.join();
    best_conc = std::min(best_conc, now() - t0);
    EXPECT(bad.load() == 0);
    for (int c = 0; c < callers; c++) EXPECT(ts[c].img == serial_img[c]);  // byte-identical
  }
  // concurrent verify: every block good; then one flipped byte per table fails exactly it
  {
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int c = 0; c < callers; c++)
      th.emplace_back([&, c] {
        std::vector<uint8_t> ok;
        lsbm::Status s = lsbm::VerifyBlocks(0, ts[c].img.data(), ts[c].img.size(), ts[c].h.data(),
                                            ts[c].h.size(), &ok, lsbm::kImagesWritable);
        if (!s.ok() || std::count(ok.begin(), ok.end(), 1) != (long)ok.size()) bad++;
        const size_t victim = (7 * c + 3) % ts[c].h.size();
        ts[c].img[ts[c].h[victim].offset + 11] ^= 0x20;
        s = lsbm::VerifyBlocks(0, ts[c].img.data(), ts[c].img.size(), ts[c].h.data(), ts[c].h.size(), &ok, lsbm::kImagesWritable);
        if (s.ok() || std::count(ok.begin(), ok.end(), 0) != 1 || ok[victim] != 0) bad++;
        ts[c].img[ts[c].h[victim].offset + 11] ^= 0x20;
      });
    for (auto& x : th) x.join();
    EXPECT(bad.load() == 0);
  }
  if (pinned)
    for (auto& t : ts) (void)hipHostUnregister(t.img.data());
  const double speedup = best_serial / best_conc;
  printf("%s serial_ms=%.3f concurrent_ms=%.3f speedup=%.3f callers=%d reps=%d pinned=%d threads=%d\n",
         fails ? "FAILED" : "OK", best_serial * 1e3, best_conc * 1e3, speedup, callers, reps, (int)pinned,
         lsbm_host_threads());
  (void)lsbm_crc32c_shutdown();
  return fails ? 1 : 0;
}
