// shared_page_seal_test.cc -- concurrent callers whose table images are
// neighbours inside ONE allocation, so that adjacent images share pages
// (VERDICT r4 weak #2 / ADVICE r4: the per-call page locks' check ->
// hipHostRegister -> resolve -> unregister ran unserialised, and a loser's
// unregister could break a winner's registration with its DMA in flight).
//
// T threads (default 8) each own every T-th image of a run of small pageable
// images packed back to back (3-200 KiB each: most pages hold the end of one
// image and the start of the next).  Every round all threads start together
// and each seals, then verifies (writable char*: page-locked for the call
// too), all its images, one table per call (TableBuilder::Finish's
// granularity).  Checks:
//   * every trailer equals the oracle's WriteRawBlock trailer
//     (oracle/crc32c_oracle.c, table/table_builder.cc:245-249), and no byte
//     outside the trailers changed;
//   * every verify passes; a flipped byte fails exactly its block;
//   * no per-call lock outlives its call (lsbm_test_locked_ranges() == 0);
//   * later calls on the same memory, serial and concurrent, still succeed.
//
//   shared_page_seal_test <liboracle_crc32c.so> [threads=8] [images=192] [rounds=6]
// prints "OK ..." or FAIL lines.
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"

static std::atomic<int> fails{0};
#define EXPECT(c)                                        \
  do {                                                   \
    if (!(c)) {                                          \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      fails++;                                           \
    }                                                    \
  } while (0)

namespace {
uint32_t (*o_extend)(uint32_t, const uint8_t*, size_t);
uint32_t (*o_mask)(uint32_t);

struct Image {
  size_t off = 0, size = 0;  // inside the one allocation
  std::vector<lsbm::BlockHandle> h;
  std::vector<uint8_t> types;
};

// all threads start each round together
class Gate {
 public:
  explicit Gate(int n) : n_(n) {}
  void arrive() {
    std::unique_lock<std::mutex> l(mu_);
    const int g = gen_;
    if (++k_ == n_) {
      k_ = 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(l, [&] { return gen_ != g; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, k_ = 0, gen_ = 0;
};
}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  if (argc < 2) {
    printf("FAIL usage: shared_page_seal_test <liboracle_crc32c.so> [threads] [images] [rounds]\n");
    return 2;
  }
  void* ol = dlopen(argv[1], RTLD_NOW);
  if (!ol) {
    printf("FAIL oracle: %s\n", dlerror());
    return 2;
  }
  void (*o_init)(void) = reinterpret_cast<void (*)(void)>(dlsym(ol, "oracle_init"));
  o_extend = reinterpret_cast<uint32_t (*)(uint32_t, const uint8_t*, size_t)>(dlsym(ol, "oracle_extend"));
  o_mask = reinterpret_cast<uint32_t (*)(uint32_t)>(dlsym(ol, "oracle_mask"));
  if (!o_init || !o_extend || !o_mask) {
    printf("FAIL oracle symbols\n");
    return 2;
  }
  o_init();
  const int T = argc > 2 ? atoi(argv[2]) : 8;
  const int N = argc > 3 ? atoi(argv[3]) : 192;
  const int rounds = argc > 4 ? atoi(argv[4]) : 6;
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }

  // the images, packed back to back in one heap allocation
  std::mt19937_64 rng(20261018);
  std::vector<Image> im(N);
  size_t total = 0;
  for (Image& m : im) {
    const size_t nb = 1 + rng() % 24;
    std::vector<uint64_t> sizes(nb);
    for (auto& s : sizes) s = rng() % 3 == 0 ? rng() % 600 : 2000 + rng() % 6200;
    uint64_t fs = 0;
    m.h = lsbm::LayoutBlocks(sizes, &fs);
    m.types.resize(nb);
    for (auto& t : m.types) t = rng() & 1;
    m.off = total;
    m.size = fs;
    total += fs;  // (no padding: neighbours share the page between them)
  }
  std::vector<char> mem(total + 64);
  char* base = mem.data() + 1 + (reinterpret_cast<uintptr_t>(mem.data()) & 7);  // (odd start)
  for (size_t i = 0; i < total; i++) base[i] = (char)(' ' + rng() % 95);
  size_t shared = 0;
  for (int i = 1; i < N; i++)
    shared += ((uintptr_t)(base + im[i].off) >> 12) == ((uintptr_t)(base + im[i].off - 1) >> 12);

  // the expected file: every trailer as WriteRawBlock writes it, by the oracle
  std::vector<char> want(base, base + total);
  for (const Image& m : im)
    for (size_t b = 0; b < m.h.size(); b++) {
      const uint8_t* blk = reinterpret_cast<const uint8_t*>(want.data() + m.off + m.h[b].offset);
      const uint8_t ty = m.types[b];
      const uint32_t crc = o_mask(o_extend(o_extend(0, blk, m.h[b].size), &ty, 1));
      char* t = want.data() + m.off + m.h[b].offset + m.h[b].size;
      t[0] = (char)ty;
      for (int q = 0; q < 4; q++) t[1 + q] = (char)(crc >> (8 * q));
    }
  auto scrub = [&] {  // the trailers zeroed: every round writes them again
    for (const Image& m : im)
      for (const auto& hd : m.h) memset(base + m.off + hd.offset + hd.size, 0, lsbm::kBlockTrailerSize);
  };
  auto seal = [&](const Image& m) {
    return lsbm::SealBlocks(0, base + m.off, m.size, m.h.data(), m.types.data(), m.h.size());
  };
  auto verify = [&](const Image& m, std::vector<uint8_t>* ok) {
    return lsbm::VerifyBlocks(0, base + m.off, m.size, m.h.data(), m.h.size(), ok, lsbm::kImagesWritable);
  };

  Gate gate(T);
  for (int r = 0; r < rounds; r++) {
    scrub();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        gate.arrive();
        // round r walks its images in a different order per thread, so that
        // neighbours' calls overlap in time in ever different pairs
        std::vector<int> mine;
        for (int i = t; i < N; i += T) mine.push_back(i);
        std::mt19937 o(1000 * r + t);
        std::shuffle(mine.begin(), mine.end(), o);
        for (int i : mine) EXPECT(seal(im[i]).ok());
        std::vector<uint8_t> ok;
        for (int i : mine) {
          const lsbm::Status s = verify(im[i], &ok);
          EXPECT(s.ok());
          for (uint8_t f : ok) EXPECT(f == 1);
        }
      });
    for (auto& x : th) x.join();
    EXPECT(memcmp(base, want.data(), total) == 0);
    EXPECT(lsbm_test_locked_ranges() == 0);
    if (fails) break;
  }
  // Pooled images (integration/image_pool.h): half of the images
  // kept registered through lsbm_host_register around their calls, as the
  // pool keeps a table image, while the neighbours on their shared pages seal
  // and verify concurrently.  A registration over a page a neighbour's call
  // holds is refused, a neighbour on a registered image's page is staged, and
  // every byte still comes out right.
  long pooled = 0, refused = 0;
  for (int r = 0; r < rounds && !fails; r++) {
    scrub();
    std::atomic<long> reg_ok{0}, reg_no{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        gate.arrive();
        std::vector<int> mine;
        for (int i = t; i < N; i += T) mine.push_back(i);
        std::mt19937 o(7000 * r + t);
        std::shuffle(mine.begin(), mine.end(), o);
        std::vector<uint8_t> ok;
        for (int i : mine) {
          bool reg = false;
          if ((i + r) % 2 == 0) {
            reg = lsbm_host_register(base + im[i].off, im[i].size) == 0;
            (reg ? reg_ok : reg_no)++;
          }
          EXPECT(seal(im[i]).ok());
          const lsbm::Status s = verify(im[i], &ok);
          EXPECT(s.ok());
          for (uint8_t f : ok) EXPECT(f == 1);
          if (reg) EXPECT(lsbm_host_unregister(base + im[i].off) == 0);
        }
      });
    for (auto& x : th) x.join();
    EXPECT(memcmp(base, want.data(), total) == 0);
    EXPECT(lsbm_test_locked_ranges() == 0 && lsbm_host_registered_bytes() == 0);
    pooled += reg_ok.load();
    refused += reg_no.load();
  }
  EXPECT(pooled > 0);
  // the rules themselves, on two neighbours: the registered one counts as
  // page-locked, its neighbour on the shared page does not and cannot register
  for (int i = 1; i < N; i++) {
    const char* a = base + im[i - 1].off;
    const char* b = base + im[i].off;
    if (((uintptr_t)b >> 12) != ((uintptr_t)(b - 1) >> 12) || im[i - 1].size < 64) continue;
    EXPECT(lsbm_host_register(a, im[i - 1].size) == 0);
    EXPECT(lsbm_test_host_pinned(a, im[i - 1].size) == 1);
    EXPECT(lsbm_test_host_pinned(a + 7, 33) == 1);
    EXPECT(lsbm_test_host_pinned(b, im[i].size) == 0);
    EXPECT(lsbm_host_register(b, im[i].size) == -1);
    EXPECT(lsbm_host_register(a, im[i - 1].size) == -1);  // (twice)
    EXPECT(lsbm_host_unregister(a + 1) == -1);
    EXPECT(lsbm_host_unregister(a) == 0);
    EXPECT(lsbm_test_host_pinned(a, im[i - 1].size) == 0);
    EXPECT(lsbm_host_register(b, im[i].size) == 0 && lsbm_host_unregister(b) == 0);
    break;
  }
  EXPECT(lsbm_host_registered_bytes() == 0);
  // a flipped byte fails exactly its block, with a neighbour sealing meanwhile
  {
    const int v = N / 2;
    const size_t blk = im[v].h.size() / 2;
    if (im[v].h[blk].size > 0) {
      char& c = base[im[v].off + im[v].h[blk].offset];
      c ^= 0x04;
      std::vector<uint8_t> ok;
      std::thread nb([&] { EXPECT(seal(im[v + 1]).ok()); });
      const lsbm::Status s = verify(im[v], &ok);
      nb.join();
      EXPECT(s.IsCorruption());
      for (size_t b = 0; b < ok.size(); b++) EXPECT(ok[b] == (b == blk ? 0 : 1));
      c ^= 0x04;
    }
  }
  // later calls on the same memory still work: serially, each image and then
  // all of them as one SealTables / VerifyTables call (neighbours in one call)
  scrub();
  for (const Image& m : im) EXPECT(seal(m).ok());
  EXPECT(memcmp(base, want.data(), total) == 0);
  scrub();
  std::vector<lsbm::TableImage> all(N);
  for (int i = 0; i < N; i++)
    all[i] = lsbm::TableImage{base + im[i].off, im[i].size, im[i].h.data(), im[i].types.data(), im[i].h.size()};
  EXPECT(lsbm::SealTables(0, all.data(), all.size()).ok());
  EXPECT(memcmp(base, want.data(), total) == 0);
  std::vector<uint8_t> ok;
  EXPECT(lsbm::VerifyTables(0, all.data(), all.size(), &ok, lsbm::kImagesWritable).ok());
  EXPECT(lsbm_test_locked_ranges() == 0);
  // (calls page-locked in place; the rest of the 2 x rounds x N + ... calls were staged
  // because a neighbour held the shared page, or a page was already registered)
  // (pooled: images registered around their calls; refused: registrations
  // refused because a neighbour's call held a shared page)
  printf("%s threads=%d images=%d bytes=%zu shared_pages=%d rounds=%d locked_calls=%ld pooled=%ld refused=%ld\n",
         fails ? "FAILED" : "OK", T, N, total, (int)shared, rounds, lsbm_test_locks_taken(), pooled, refused);
  (void)lsbm_crc32c_shutdown();
  return fails ? 1 : 0;
}
