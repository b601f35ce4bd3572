// bench_host_layers.cc -- host -> host rates of the C++ layers (GPU box).
//
//   include/lsbm/table_checksum.h  SealBlocks / VerifyBlocks on one 16 MiB
//                                  table; SealTables / VerifyTables on a
//                                  compaction's worth of 16 MiB tables
//   include/lsbm/log_checksum.h    BatchWriter::Seal of a ~1 GB WAL (one group
//                                  commit) and BatchReader Verify + replay
// against the PCIe ceiling measured in the same run: a plain hipMemcpy of the
// same bytes from pinned memory.  Tables are db_bench-shaped (4,118-B data
// blocks with trailers, printable bytes); every sealed table is re-checked
// on a sample of blocks against util/crc32c.h (the library's scalar API).
//
//   build: g++ -O2 -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//          tools/bench_host_layers.cc -Llsbm_amd -llsbm_crc32c \
//          -Wl,-rpath,lsbm_amd -lamdhip64 -L/opt/rocm/lib -pthread -o build/bench_host_layers
//   run:   build/bench_host_layers [tables=1000] [wal_mb=1024]
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <sys/resource.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "lsbm/log_checksum.h"
#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"
#include "util/crc32c.h"

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// this process's CPU time, every thread (the caller, the pool, HIP's own)
double cpu_s() {
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void fill_printable(char* p, size_t n, uint64_t seed) {
  const unsigned nt = 16;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++)
    th.emplace_back([=] {
      const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
      uint64_t x = seed * 1000003 + t;
      for (size_t i = lo; i < hi; i += 8) {
        uint64_t r = splitmix(x);
        for (int k = 0; k < 8 && i + k < hi; k++, r >>= 8) p[i + k] = (char)(' ' + (r & 0xff) % 95);
      }
    });
  for (auto& t : th) t.join();
}

struct Table {
  std::vector<char> img;
  std::vector<lsbm::BlockHandle> h;
  std::vector<uint8_t> types;
};

// a 16 MiB table of 4,118-B data blocks (the db_bench mode)
void make_table(Table* t, uint64_t seed, size_t bytes) {
  const size_t per = 4118 + lsbm::kBlockTrailerSize;
  const size_t n = bytes / per;
  uint64_t fs = 0;
  t->h = lsbm::LayoutBlocks(std::vector<uint64_t>(n, 4118), &fs);
  t->img.assign(fs, 0);
  fill_printable(t->img.data(), fs, seed);
  t->types.assign(n, 0);
}

int check_table(const Table& t, size_t stride) {
  int bad = 0;
  for (size_t i = 0; i < t.h.size(); i += stride) {
    const char* b = t.img.data() + t.h[i].offset;
    uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(b, t.h[i].size), b + t.h[i].size, 1);
    uint32_t stored;
    memcpy(&stored, b + t.h[i].size + 1, 4);
    bad += leveldb::crc32c::Unmask(stored) != crc;
  }
  return bad;
}

}  // namespace

int main(int argc, char** argv) {
  const size_t ntables = argc > 1 ? strtoul(argv[1], nullptr, 10) : 1000;
  const size_t wal_mb = argc > 2 ? strtoul(argv[2], nullptr, 10) : 1024;
  const size_t kTable = 16u << 20;
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    fprintf(stderr, "no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  // ---- PCIe ceiling: pinned H2D of 1 GiB ----
  {
    const size_t n = 1u << 30;
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess || hipMalloc(&d, n) != hipSuccess) {
      fprintf(stderr, "h2d ceiling: allocation failed\n");
      return 1;
    }
    memset(h, 1, n);
    bool ok = hipMemcpy(d, h, n, hipMemcpyHostToDevice) == hipSuccess;
    double t0 = now();
    for (int r = 0; r < 3; r++) ok = ok && hipMemcpy(d, h, n, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
      fprintf(stderr, "h2d ceiling: copy failed\n");
      return 1;
    }
    const double el = (now() - t0) / 3;
    printf("{\"what\": \"h2d_pinned_copy\", \"bytes\": %zu, \"GBps\": %.2f}\n", n, n / el / 1e9);
    (void)hipHostFree(h);
    (void)hipFree(d);
  }
  // ---- one 16 MiB table ----
  {
    Table t;
    make_table(&t, 1, kTable);
    lsbm::Status s = lsbm::SealBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.types.data(), t.h.size());
    // per-call times: the mean, and the median (a call now and then takes
    // ~15 ms more, in the runtime, outside the layer's copy / wait / results)
    const int reps = 20;
    std::vector<double> ts, tv;
    double c0 = cpu_s();
    for (int r = 0; r < reps && s.ok(); r++) {
      const double t0 = now();
      s = lsbm::SealBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.types.data(), t.h.size());
      ts.push_back(now() - t0);
    }
    const double cpu_seal = (cpu_s() - c0) / reps;
    std::vector<uint8_t> ok;
    c0 = cpu_s();
    for (int r = 0; r < reps && s.ok(); r++) {
      const double t0 = now();
      s = lsbm::VerifyBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.h.size(), &ok, lsbm::kImagesWritable);
      tv.push_back(now() - t0);
    }
    const double cpu_verify = (cpu_s() - c0) / reps;
    auto mean = [](const std::vector<double>& v) {
      double a = 0;
      for (double x : v) a += x;
      return v.empty() ? 0.0 : a / v.size();
    };
    auto median = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      return v.empty() ? 0.0 : v[v.size() / 2];
    };
    const double el_s = median(ts), el_v = median(tv);
    printf("{\"what\": \"one_table_16MiB\", \"blocks\": %zu, \"status\": \"%s\", \"seal_ms\": %.3f, "
           "\"seal_GBps\": %.2f, \"verify_ms\": %.3f, \"verify_GBps\": %.2f, \"seal_mean_ms\": %.3f, "
           "\"verify_mean_ms\": %.3f, \"seal_cpu_ms_per_call\": %.3f, \"verify_cpu_ms_per_call\": %.3f, "
           "\"sample_bad\": %d}\n",
           t.h.size(), s.ToString().c_str(), el_s * 1e3, t.img.size() / el_s / 1e9, el_v * 1e3,
           t.img.size() / el_v / 1e9, mean(ts) * 1e3, mean(tv) * 1e3, cpu_seal * 1e3, cpu_verify * 1e3,
           check_table(t, 7));
  }
  // ---- a compaction: ntables x 16 MiB, pageable and page-locked ----
  {
    std::vector<Table> ts(ntables);
    for (size_t i = 0; i < ntables; i++) make_table(&ts[i], 100 + i, kTable);
    std::vector<lsbm::TableImage> im(ntables);
    size_t bytes = 0;
    for (size_t i = 0; i < ntables; i++) {
      im[i] = lsbm::TableImage{ts[i].img.data(), ts[i].img.size(), ts[i].h.data(), ts[i].types.data(),
                               ts[i].h.size()};
      bytes += ts[i].img.size();
    }
    for (int pinned = 0; pinned < 2; pinned++) {
      if (pinned)
        for (auto& t : ts)
          if (hipHostRegister(t.img.data(), t.img.size(), hipHostRegisterDefault) != hipSuccess) {
            fprintf(stderr, "hipHostRegister failed\n");
            return 1;
          }
      // warm at the timed size: the session's stages grow to 64 MiB chunks once
      lsbm::Status s = lsbm::SealTables(0, im.data(), ntables);
      double t0 = now(), c0 = cpu_s();
      s = lsbm::SealTables(0, im.data(), ntables);
      const double el_s = now() - t0, cpu_seal = cpu_s() - c0;
      int bad = 0;
      for (size_t i = 0; i < ntables; i += 37) bad += check_table(ts[i], 13);
      std::vector<uint8_t> ok;
      t0 = now();
      c0 = cpu_s();
      lsbm::Status v = lsbm::VerifyTables(0, im.data(), ntables, &ok);
      const double el_v = now() - t0, cpu_verify = cpu_s() - c0;
      size_t nok = 0;
      for (uint8_t o : ok) nok += o;
      printf("{\"what\": \"compaction_tables\", \"tables\": %zu, \"bytes\": %zu, \"pinned\": %d, "
             "\"seal\": \"%s\", \"seal_s\": %.3f, \"seal_GBps\": %.2f, \"verify\": \"%s\", \"verify_s\": %.3f, "
             "\"verify_GBps\": %.2f, \"seal_cpu_ms_per_table\": %.3f, \"verify_cpu_ms_per_table\": %.3f, "
             "\"blocks_ok\": %zu, \"blocks\": %zu, \"sample_bad\": %d}\n",
             ntables, bytes, pinned, s.ToString().c_str(), el_s, bytes / el_s / 1e9, v.ToString().c_str(),
             el_v, bytes / el_v / 1e9, cpu_seal * 1e3 / ntables, cpu_verify * 1e3 / ntables, nok, ok.size(), bad);
      if (pinned)
        for (auto& t : ts) (void)hipHostUnregister(t.img.data());
    }
  }
  // ---- a WAL: one group commit of ~wal_mb MiB, then recovery's read ----
  {
    std::vector<char> payload(wal_mb << 20);
    fill_printable(payload.data(), payload.size(), 7);
    // two writers with the same records: the first group commit warms the
    // session's staging for this shape (its buffers grow to the largest
    // window's header count once), the second is timed
    lsbm::log::BatchWriter warm, w;
    size_t nrec = 0;
    for (lsbm::log::BatchWriter* bw : {&warm, &w}) {
      uint64_t x = 99;
      size_t pos = 0;
      nrec = 0;
      while (pos < payload.size()) {  // db_bench-like records, mean ~1270 B
        const size_t len = std::min<size_t>(splitmix(x) % 2541, payload.size() - pos);
        bw->AddRecord(payload.data() + pos, len);
        pos += len;
        nrec++;
      }
    }
    lsbm::Status s = warm.Seal(0);
    double t0 = now(), c0 = cpu_s();
    if (s.ok()) s = w.Seal(0);
    const double el_s = now() - t0, cpu_seal = cpu_s() - c0;
    const std::string& img = w.contents();
    struct Count : lsbm::log::Reporter {
      size_t drops = 0;
      void Corruption(size_t, const lsbm::Status&) override { drops++; }
    } rep;
    t0 = now();
    c0 = cpu_s();
    lsbm::log::BatchReader r(img.data(), img.size(), &rep);
    lsbm::Status v = r.Verify(0);
    const double el_v = now() - t0, cpu_verify = cpu_s() - c0;
    std::string rec;
    size_t got = 0;
    t0 = now();
    while (r.ReadRecord(&rec)) got++;
    const double el_r = now() - t0;
    printf("{\"what\": \"wal\", \"bytes\": %zu, \"records\": %zu, \"physical\": %zu, \"seal\": \"%s\", "
           "\"seal_s\": %.3f, \"seal_GBps\": %.2f, \"verify\": \"%s\", \"verify_s\": %.3f, \"verify_GBps\": %.2f, "
           "\"replay_s\": %.3f, \"seal_cpu_ms_per_GB\": %.2f, \"verify_cpu_ms_per_GB\": %.2f, "
           "\"records_read\": %zu, \"drops\": %zu}\n",
           img.size(), nrec, w.headers().size(), s.ToString().c_str(), el_s, img.size() / el_s / 1e9,
           v.ToString().c_str(), el_v, img.size() / el_v / 1e9, el_r, cpu_seal * 1e3 / (img.size() / 1e9),
           cpu_verify * 1e3 / (img.size() / 1e9), got, rep.drops);
  }
  return lsbm_crc32c_shutdown() == LSBM_OK ? 0 : 1;
}
