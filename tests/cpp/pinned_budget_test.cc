// pinned_budget_test.cc -- the C++ layers' page-locked staging stays bounded
// per device (up to 8 sessions x 4 stages of staging, ~2.5 GiB of
// pinned memory per device held until shutdown).  Run with a small
// LSBM_PINNED_MB and LSBM_AUTO_LOCK=0 (so every call stages through the
// session's pinned buffers): C threads seal and verify their own 16 MiB tables
// at once (each leases its own session), then the pinned bytes held by the
// device's sessions must have come back under the budget plus one session's
// worth (a released lease frees the other idle sessions' staging), and later
// calls, which grow the buffers again, must still be correct.
//
//   pinned_budget_test [callers=6] [budget_mb]   prints "OK ..." or FAIL lines
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"
#include "util/crc32c.h"

static std::atomic<int> fails{0};
#define EXPECT(c)                                        \
  do {                                                   \
    if (!(c)) {                                          \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      fails++;                                           \
    }                                                    \
  } while (0)

namespace {
struct Table {
  std::vector<char> img;
  std::vector<lsbm::BlockHandle> h;
  std::vector<uint8_t> types;
};

void make_table(Table* t, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<uint64_t> sizes((16u << 20) / 4123);
  for (auto& s : sizes) s = 3900 + rng() % 400;
  uint64_t fs = 0;
  t->h = lsbm::LayoutBlocks(sizes, &fs);
  t->img.assign(fs, 0);
  for (auto& c : t->img) c = (char)(' ' + rng() % 95);
  t->types.assign(sizes.size(), 0);
}

bool trailers_ok(const Table& t) {
  for (size_t i = 0; i < t.h.size(); i++) {
    const char* b = t.img.data() + t.h[i].offset;
    const char type = (char)t.types[i];
    const uint32_t m = leveldb::crc32c::Mask(leveldb::crc32c::Extend(leveldb::crc32c::Value(b, t.h[i].size), &type, 1));
    char want[5] = {type, (char)m, (char)(m >> 8), (char)(m >> 16), (char)(m >> 24)};
    if (memcmp(want, b + t.h[i].size, 5) != 0) return false;
  }
  return true;
}
}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int callers = argc > 1 ? atoi(argv[1]) : 6;
  const char* env = getenv("LSBM_PINNED_MB");
  const unsigned long long budget = (unsigned long long)(env ? atol(env) : 1024) << 20;
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  std::vector<Table> ts(callers);
  for (int c = 0; c < callers; c++) make_table(&ts[c], 500 + c);
  unsigned long long peak = 0, one_session = 0;
  for (int round = 0; round < 3; round++) {
    std::vector<std::thread> th;
    std::atomic<unsigned long long> seen{0};
    for (int c = 0; c < callers; c++)
      th.emplace_back([&, c] {
        for (auto& hd : ts[c].h) memset(ts[c].img.data() + hd.offset + hd.size, 0, 5);
        EXPECT(lsbm::SealBlocks(0, ts[c].img.data(), ts[c].img.size(), ts[c].h.data(), ts[c].types.data(),
                                ts[c].h.size())
                   .ok());
        std::vector<uint8_t> ok;
        EXPECT(lsbm::VerifyBlocks(0, ts[c].img.data(), ts[c].img.size(), ts[c].h.data(), ts[c].h.size(), &ok, lsbm::kImagesWritable).ok());
        unsigned long long b = lsbm_test_pinned_bytes(0), m = seen.load();
        while (b > m && !seen.compare_exchange_weak(m, b)) {
        }
      });
    for (auto& x : th) x.join();
    for (int c = 0; c < callers; c++) EXPECT(trailers_ok(ts[c]));
    peak = std::max(peak, seen.load());
    const unsigned long long after = lsbm_test_pinned_bytes(0);
    const int sessions = lsbm_test_session_count(0);
    if (round == 0) one_session = sessions ? peak / sessions : peak;
    // every lease is released: at most the budget plus the session released last
    EXPECT(after <= budget + one_session + (4u << 20));
    printf("round %d: sessions=%d peak_pinned_MiB=%.1f after_MiB=%.1f\n", round, sessions, peak / 1048576.0,
           after / 1048576.0);
  }
  printf("%s callers=%d budget_MiB=%llu peak_MiB=%.1f\n", fails ? "FAILED" : "OK", callers, budget >> 20,
         peak / 1048576.0);
  (void)lsbm_crc32c_shutdown();
  EXPECT(lsbm_test_pinned_bytes(0) == 0);  // (shutdown freed everything)
  return fails ? 1 : 0;
}
