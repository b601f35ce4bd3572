// bench_one_table.cc -- the reference's own call granularity for the table
// layer: one 16 MiB table per SealBlocks / VerifyBlocks call, as
// TableBuilder::Finish would make it (lsbm/db_impl.cc:843-892 finishes one
// output table at a time), timed call by call.
//
// Prints one JSON line per phase with the per-call distribution (p50 / p90 /
// p99 / max / mean, the slowest calls' indices) and the cgroup CPU throttling
// counters (/sys/fs/cgroup/cpu.stat: nr_periods, nr_throttled,
// throttled_usec) read before and after the phase:
//   host_copy_*                           the pageable layers' staging copy alone
//   seal_pageable, verify_pageable        reps calls each, back to back
//   alternate_pageable                    seal, verify, seal, ... (reps each)
//   seal_register_per_call                hipHostRegister + seal + unregister
//   seal_locked, verify_locked            the same image hipHostRegister'ed
//   zerocopy_*, dma_*                     the device ABI on the registered image
//                                         in place, and the DMA path's floor
//   concurrent_seal                       C caller threads, each sealing its
//                                         own table reps / C times, against the
//                                         same calls made one after another
//
//   build: make -C tools bench_one_table
//   run:   build/bench_one_table [reps=100] [callers=4] [table_mib=16] [idle_ms=0]
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "lsbm/table_checksum.h"
#include "lsbm_crc32c.h"
#include "util/crc32c.h"

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double g_t_first = 0;  // the first layer call of the process (set by main)

uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Table {
  std::vector<char> img;
  std::vector<lsbm::BlockHandle> h;
  std::vector<uint8_t> types;
};

// db_bench-shaped: 4,118-B data blocks with trailers, printable bytes
void make_table(Table* t, uint64_t seed, size_t bytes) {
  const size_t n = bytes / (4118 + lsbm::kBlockTrailerSize);
  uint64_t fs = 0;
  t->h = lsbm::LayoutBlocks(std::vector<uint64_t>(n, 4118), &fs);
  t->img.assign(fs, 0);
  uint64_t x = seed;
  for (size_t i = 0; i < fs; i += 8) {
    uint64_t r = splitmix(x);
    for (size_t k = 0; k < 8 && i + k < fs; k++, r >>= 8) t->img[i + k] = (char)(' ' + (r & 0xff) % 95);
  }
  t->types.assign(n, 0);
}

int check_table(const Table& t) {
  int bad = 0;
  for (size_t i = 0; i < t.h.size(); i++) {
    const char* b = t.img.data() + t.h[i].offset;
    const uint32_t crc = leveldb::crc32c::Extend(leveldb::crc32c::Value(b, t.h[i].size), b + t.h[i].size, 1);
    uint32_t stored;
    memcpy(&stored, b + t.h[i].size + 1, 4);
    bad += leveldb::crc32c::Unmask(stored) != crc;
  }
  return bad;
}

struct CpuStat {
  long long periods = -1, throttled = -1, throttled_us = -1, usage_us = -1;
  double proc_s = 0;  // this process's CPU time, all threads (getrusage)
};
double proc_cpu_s() {
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}
CpuStat read_cpu_stat() {
  CpuStat c;
  c.proc_s = proc_cpu_s();
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return c;
  char key[64];
  long long v;
  while (fscanf(f, "%63s %lld", key, &v) == 2) {
    if (!strcmp(key, "nr_periods")) c.periods = v;
    else if (!strcmp(key, "nr_throttled")) c.throttled = v;
    else if (!strcmp(key, "throttled_usec")) c.throttled_us = v;
    else if (!strcmp(key, "usage_usec")) c.usage_us = v;
  }
  fclose(f);
  return c;
}

std::string dist_json(std::vector<double> v, double bytes) {
  if (v.empty()) return "{}";
  std::vector<size_t> idx(v.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return v[a] > v[b]; });
  double mean = 0;
  for (double x : v) mean += x;
  mean /= v.size();
  std::vector<double> s = v;
  std::sort(s.begin(), s.end());
  auto q = [&](double p) { return s[std::min(s.size() - 1, (size_t)(p * (s.size() - 1) + 0.5))]; };
  char buf[1024];
  std::string slow;
  for (size_t k = 0; k < std::min<size_t>(5, idx.size()); k++) {
    char t[64];
    snprintf(t, sizeof(t), "%s[%zu, %.3f]", k ? ", " : "", idx[k], v[idx[k]] * 1e3);
    slow += t;
  }
  snprintf(buf, sizeof(buf),
           "{\"calls\": %zu, \"p50_ms\": %.3f, \"p90_ms\": %.3f, \"p99_ms\": %.3f, \"max_ms\": %.3f, "
           "\"mean_ms\": %.3f, \"min_ms\": %.3f, \"p50_GBps\": %.2f, \"p99_over_p50\": %.2f, \"slowest\": [%s]}",
           v.size(), q(0.5) * 1e3, q(0.9) * 1e3, q(0.99) * 1e3, s.back() * 1e3, mean * 1e3, s.front() * 1e3,
           bytes / q(0.5) / 1e9, q(0.99) / q(0.5), slow.c_str());
  return buf;
}

void print_phase(const char* what, const std::vector<double>& v, double bytes, const CpuStat& a,
                 const CpuStat& b, const char* status, int bad, const std::vector<double>& starts = {}) {
  double slow_at = -1;  // the slowest call's start, ms after the process's first layer call
  if (!starts.empty())
    slow_at = (starts[std::max_element(v.begin(), v.end()) - v.begin()] - g_t_first) * 1e3;
  // host CPU per call: this process's CPU time (every thread: the caller,
  // the pool's workers, HIP's own) over the phase, divided by its calls
  printf("{\"what\": \"%s\", \"bytes\": %.0f, \"dist\": %s, \"slowest_at_ms\": %.1f, "
         "\"host_cpu_ms_per_call\": %.3f, \"cpu_stat\": {\"nr_periods\": %lld, "
         "\"nr_throttled\": %lld, \"throttled_ms\": %.3f, \"cpu_ms\": %.1f}, \"status\": \"%s\", \"bad\": %d}\n",
         what, bytes, dist_json(v, bytes).c_str(), slow_at, v.empty() ? 0.0 : (b.proc_s - a.proc_s) * 1e3 / v.size(),
         b.periods - a.periods, b.throttled - a.throttled, (b.throttled_us - a.throttled_us) / 1e3,
         (b.usage_us - a.usage_us) / 1e3, status, bad);
  fflush(stdout);
}

// A CPU-bound co-runner's unit of work: xorshift steps (no memory traffic).
uint64_t spin_work(uint64_t iters, uint64_t seed) {
  uint64_t x = seed | 1;
  for (uint64_t i = 0; i < iters; i++) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
  }
  return x;
}
double thread_cpu_s() {
  struct rusage ru;
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}
int usable_cores_guess() { return lsbm_host_threads() + 1; }
volatile uint64_t g_sink;

// k co-runner threads each do a fixed amount of CPU-bound work (calibrated to
// ~ the time of 100 calls), alone and then while this thread makes layer
// calls back to back; prints the co-runners' slowdown and the layer's own
// host CPU per call (the process's CPU time less the co-runners').
void corunner_phase(const char* what, const std::function<lsbm::Status()>& call, int k) {
  // the call's time, and the work that takes 100 of them on one core
  const double c0 = now();
  for (int i = 0; i < 10; i++) (void)call();
  const double per_call = (now() - c0) / 10;
  const double w0 = now();
  g_sink = spin_work(20000000, 1);
  const double per_iter = (now() - w0) / 20000000;
  const uint64_t iters = (uint64_t)(100 * per_call / per_iter);
  auto run_corunners = [&](bool beside, double* wall_max, double* cpu_sum, int* calls) {
    std::atomic<int> left{k};
    std::vector<double> wall(k), cpu(k);
    std::vector<std::thread> th;
    std::atomic<bool> go{false};
    for (int j = 0; j < k; j++)
      th.emplace_back([&, j] {
        while (!go.load()) std::this_thread::yield();
        const double t0 = now(), u0 = thread_cpu_s();
        g_sink = spin_work(iters, j + 2);
        wall[j] = now() - t0;
        cpu[j] = thread_cpu_s() - u0;
        left--;
      });
    go.store(true);
    int n = 0;
    if (beside)
      while (left.load() > 0) {
        (void)call();
        n++;
      }
    for (auto& x : th) x.join();
    *wall_max = *std::max_element(wall.begin(), wall.end());
    *cpu_sum = 0;
    for (double c : cpu) *cpu_sum += c;
    *calls = n;
  };
  std::vector<double> alone, beside, layer_cpu;
  int calls = 0;
  for (int rep = 0; rep < 5; rep++) {
    double wmax, csum;
    int n;
    run_corunners(false, &wmax, &csum, &n);
    alone.push_back(wmax);
    const double p0 = proc_cpu_s();
    run_corunners(true, &wmax, &csum, &n);
    beside.push_back(wmax);
    layer_cpu.push_back(n ? (proc_cpu_s() - p0 - csum) / n : 0.0);
    calls += n;
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("{\"what\": \"corunner_%s\", \"corunner_threads\": %d, \"call_ms\": %.3f, \"alone_ms\": %.2f, "
         "\"beside_ms\": %.2f, \"slowdown_pct\": %.2f, \"calls\": %d, \"layer_cpu_ms_per_call\": %.3f, "
         "\"pool_threads\": %d}\n",
         what, k, per_call * 1e3, med(alone) * 1e3, med(beside) * 1e3, 100 * (med(beside) / med(alone) - 1), calls,
         med(layer_cpu) * 1e3, lsbm_host_threads());
  fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 100;
  const int callers = argc > 2 ? atoi(argv[2]) : 4;
  const size_t mib = argc > 3 ? strtoul(argv[3], nullptr, 10) : 16;
  const int idle_ms = argc > 4 ? atoi(argv[4]) : 0;  // pause after the warm-up calls
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    fprintf(stderr, "no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  Table t;
  make_table(&t, 1, mib << 20);
  const double bytes = (double)t.img.size();
  lsbm::Status s;
  std::vector<uint8_t> ok;
  // warm: the session's staging for this shape, the pool's threads
  g_t_first = now();
  for (int r = 0; r < 3; r++) {
    s = lsbm::SealBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.types.data(), t.h.size());
    if (s.ok()) s = lsbm::VerifyBlocks(0, t.img.data(), t.img.size(), t.h.data(), t.h.size(), &ok, lsbm::kImagesWritable);
  }
  if (!s.ok()) {
    fprintf(stderr, "warm-up: %s\n", s.ToString().c_str());
    return 1;
  }
  if (idle_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(idle_ms));
  auto seal = [&](Table& tb) {
    return lsbm::SealBlocks(0, tb.img.data(), tb.img.size(), tb.h.data(), tb.types.data(), tb.h.size());
  };
  auto verify = [&](Table& tb) {
    return lsbm::VerifyBlocks(0, tb.img.data(), tb.img.size(), tb.h.data(), tb.h.size(), &ok, lsbm::kImagesWritable);
  };
  auto phase = [&](const char* what, const std::function<lsbm::Status()>& call) {
    std::vector<double> v, starts;
    const CpuStat a = read_cpu_stat();
    lsbm::Status st;
    for (int r = 0; r < reps && st.ok(); r++) {
      const double t0 = now();
      st = call();
      v.push_back(now() - t0);
      starts.push_back(t0);
    }
    const CpuStat b = read_cpu_stat();
    print_phase(what, v, bytes, a, b, st.ToString().c_str(), check_table(t), starts);
    return st.ok();
  };
  {
    // The pageable layers' staging copy alone (the pageable seal's critical
    // path): the table into a page-locked buffer over the pool, one chunk's
    // worth over the pool, and on one thread.
    void* stg = nullptr;
    if (hipHostMalloc(&stg, t.img.size(), hipHostMallocDefault) == hipSuccess) {
      auto copy_phase = [&](const char* what, size_t n, int par) {
        std::vector<double> v;
        for (int r = 0; r < reps; r++) {
          const double t0 = now();
          lsbm_test_host_copy(stg, t.img.data(), n, par);
          v.push_back(now() - t0);
        }
        printf("{\"what\": \"%s\", \"bytes\": %zu, \"threads\": %d, \"dist\": %s}\n", what, n,
               par ? lsbm_host_threads() + 1 : 1, dist_json(v, (double)n).c_str());
      };
      copy_phase("host_copy_table_pool", t.img.size(), 1);
      copy_phase("host_copy_4MiB_pool", std::min<size_t>(t.img.size(), 4u << 20), 1);
      copy_phase("host_copy_table_one_thread", t.img.size(), 0);
      (void)hipHostFree(stg);
    }
  }
  for (int locked = 0; locked < 2; locked++) {
    if (locked && hipHostRegister(t.img.data(), t.img.size(), hipHostRegisterDefault) != hipSuccess) {
      fprintf(stderr, "hipHostRegister failed\n");
      return 1;
    }
    const std::string sfx = locked ? "_locked" : "_pageable";
    if (getenv("LSBM_BENCH_VERIFY_FIRST")) {  // (order effects: verify, seal, verify again)
      if (!phase(("verify" + sfx).c_str(), [&] { return verify(t); })) return 1;
      if (!phase(("seal" + sfx).c_str(), [&] { return seal(t); })) return 1;
      if (!phase(("verify_again" + sfx).c_str(), [&] { return verify(t); })) return 1;
    } else {
      if (!phase(("seal" + sfx).c_str(), [&] { return seal(t); })) return 1;
      if (!phase(("verify" + sfx).c_str(), [&] { return verify(t); })) return 1;
    }
    if (!locked) {
      // The same bytes as const char* (a read-only mapping, for all the layer
      // knows): staged through pinned buffers; and what the layer's calls cost
      // a CPU-bound co-runner.
      auto verify_const = [&](Table& tb) {
        return lsbm::VerifyBlocks(0, static_cast<const char*>(tb.img.data()), tb.img.size(), tb.h.data(),
                                  tb.h.size(), &ok);
      };
      if (!phase("verify_pageable_const_staged", [&] { return verify_const(t); })) return 1;
      corunner_phase("verify_const_staged", [&] { return verify_const(t); }, 1);
      corunner_phase("verify_heap_locked", [&] { return verify(t); }, 1);
      corunner_phase("seal_pageable_locked", [&] { return seal(t); }, 1);
      const int all_but_one = std::max(1, usable_cores_guess() - 1);
      corunner_phase("verify_const_staged", [&] { return verify_const(t); }, all_but_one);
      corunner_phase("verify_heap_locked", [&] { return verify(t); }, all_but_one);
      corunner_phase("seal_pageable_locked", [&] { return seal(t); }, all_but_one);
    }
    if (!locked) {
      // seal and verify alternating: is the seal's tail the order it runs in?
      std::vector<double> vs, vv;
      const CpuStat a = read_cpu_stat();
      for (int r = 0; r < reps && s.ok(); r++) {
        double t0 = now();
        s = seal(t);
        vs.push_back(now() - t0);
        t0 = now();
        if (s.ok()) s = verify(t);
        vv.push_back(now() - t0);
      }
      const CpuStat b = read_cpu_stat();
      print_phase("alternate_seal_pageable", vs, bytes, a, b, s.ToString().c_str(), check_table(t));
      print_phase("alternate_verify_pageable", vv, bytes, a, b, s.ToString().c_str(), 0);
      if (!s.ok()) return 1;
    }
    if (!locked) {
      // page-locking the image for each call (hipHostRegister, seal,
      // hipHostUnregister): what a caller that does not keep its write buffer
      // registered would pay; and the registration alone, on this image
      // (std::vector: transparent huge pages where the system gives them) and
      // on a copy in 4 KiB pages (MADV_NOHUGEPAGE)
      auto reg_seal = [&](Table& tb) {
        if (hipHostRegister(tb.img.data(), tb.img.size(), hipHostRegisterDefault) != hipSuccess)
          return lsbm::Status::IOError("hipHostRegister");
        lsbm::Status r = seal(tb);
        (void)hipHostUnregister(tb.img.data());
        return r;
      };
      auto reg_only = [&](void* p, size_t n) {
        if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) return lsbm::Status::IOError("register");
        return hipHostUnregister(p) == hipSuccess ? lsbm::Status::OK() : lsbm::Status::IOError("unregister");
      };
      if (!phase("seal_register_per_call", [&] { return reg_seal(t); })) return 1;
      if (!phase("register_unregister_only", [&] { return reg_only(t.img.data(), t.img.size()); })) return 1;
      const size_t n4 = (t.img.size() + 4095) & ~(size_t)4095;
      void* m4 = mmap(nullptr, n4, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m4 != MAP_FAILED) {
        (void)madvise(m4, n4, MADV_NOHUGEPAGE);
        memcpy(m4, t.img.data(), t.img.size());
        if (!phase("register_unregister_only_4k_pages", [&] { return reg_only(m4, t.img.size()); })) return 1;
        if (!phase("seal_register_per_call_4k_pages", [&] {
              if (hipHostRegister(m4, t.img.size(), hipHostRegisterDefault) != hipSuccess)
                return lsbm::Status::IOError("hipHostRegister");
              lsbm::Status r = lsbm::SealBlocks(0, static_cast<char*>(m4), t.img.size(), t.h.data(), t.types.data(),
                                                t.h.size());
              (void)hipHostUnregister(m4);
              return r;
            }))
          return 1;
        if (!phase("seal_pageable_4k_pages", [&] {
              return lsbm::SealBlocks(0, static_cast<char*>(m4), t.img.size(), t.h.data(), t.types.data(),
                                      t.h.size());
            }))
          return 1;
        munmap(m4, n4);
      }
    }
    if (locked) {
      // Zero-copy experiment: the device ABI's kernels reading the registered
      // image over PCIe directly (no DMA, no staging), handles and results in
      // device memory: is a kernel's own PCIe read stream faster per table
      // than DMA + kernel?
      void* dimg = nullptr;
      uint64_t* dh = nullptr;
      uint8_t *dt = nullptr, *dok = nullptr;
      uint32_t* dm = nullptr;
      hipStream_t st = nullptr;
      std::vector<uint64_t> hh(2 * t.h.size());
      for (size_t i = 0; i < t.h.size(); i++) hh[2 * i] = t.h[i].offset, hh[2 * i + 1] = t.h[i].size;
      bool ok_setup = hipHostGetDevicePointer(&dimg, t.img.data(), 0) == hipSuccess &&
                      hipMalloc(reinterpret_cast<void**>(&dh), hh.size() * 8) == hipSuccess &&
                      hipMalloc(reinterpret_cast<void**>(&dt), t.h.size()) == hipSuccess &&
                      hipMalloc(reinterpret_cast<void**>(&dok), t.h.size()) == hipSuccess &&
                      hipMalloc(reinterpret_cast<void**>(&dm), t.h.size() * 4) == hipSuccess &&
                      hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
                      hipMemcpy(dh, hh.data(), hh.size() * 8, hipMemcpyHostToDevice) == hipSuccess &&
                      hipMemcpy(dt, t.types.data(), t.h.size(), hipMemcpyHostToDevice) == hipSuccess;
      if (ok_setup) {
        auto zc = [&](bool seal_mode) {
          const int rc = seal_mode ? lsbm_sst_trailer_crcs_dev(static_cast<const uint8_t*>(dimg), t.img.size(), dh,
                                                               dt, t.h.size(), dm, nullptr, st)
                                   : lsbm_sst_verify_dev(static_cast<const uint8_t*>(dimg), t.img.size(), dh,
                                                         t.h.size(), dok, nullptr, st);
          const bool good = rc == LSBM_OK && hipStreamSynchronize(st) == hipSuccess;
          return good ? lsbm::Status::OK() : lsbm::Status::IOError("zero-copy launch");
        };
        for (int w = 0; w < 3; w++) (void)zc(false);
        if (!phase("zerocopy_trailer_crcs_locked", [&] { return zc(true); })) return 1;
        if (!phase("zerocopy_verify_locked", [&] { return zc(false); })) return 1;
        std::vector<uint8_t> okh(t.h.size());
        (void)hipMemcpy(okh.data(), dok, okh.size(), hipMemcpyDeviceToHost);
        printf("{\"what\": \"zerocopy_check\", \"blocks_ok\": %zu, \"blocks\": %zu}\n",
               (size_t)std::count(okh.begin(), okh.end(), 1), okh.size());
        // The DMA path's floor: the table's bytes alone over the copy engines,
        // from this registered image and from a hipHostMalloc'd one, whole or
        // in 4 chunks on one stream, and whole + the verify kernel behind it.
        void* dbuf = nullptr;
        void* hm = nullptr;
        if (hipMalloc(&dbuf, t.img.size()) == hipSuccess &&
            hipHostMalloc(&hm, t.img.size(), hipHostMallocDefault) == hipSuccess) {
          memcpy(hm, t.img.data(), t.img.size());
          auto dma = [&](const void* src, int pieces, bool kernel) {
            const size_t n = t.img.size(), step = (n + pieces - 1) / pieces;
            bool good = true;
            for (size_t o = 0; o < n && good; o += step)
              good = hipMemcpyAsync(static_cast<char*>(dbuf) + o, static_cast<const char*>(src) + o,
                                    std::min(step, n - o), hipMemcpyHostToDevice, st) == hipSuccess;
            if (good && kernel)
              good = lsbm_sst_verify_dev(static_cast<const uint8_t*>(dbuf), n, dh, t.h.size(), dok, nullptr, st) ==
                     LSBM_OK;
            good = good && hipStreamSynchronize(st) == hipSuccess;
            return good ? lsbm::Status::OK() : lsbm::Status::IOError("dma");
          };
          for (int w = 0; w < 3; w++) (void)dma(hm, 1, true);
          if (!phase("dma_only_registered", [&] { return dma(t.img.data(), 1, false); })) return 1;
          if (!phase("dma_only_registered_4", [&] { return dma(t.img.data(), 4, false); })) return 1;
          if (!phase("dma_only_hostmalloc", [&] { return dma(hm, 1, false); })) return 1;
          if (!phase("dma_verify_registered", [&] { return dma(t.img.data(), 1, true); })) return 1;
          if (!phase("dma_verify_hostmalloc", [&] { return dma(hm, 1, true); })) return 1;
        } else {
          printf("{\"what\": \"dma_only\", \"status\": \"setup failed\"}\n");
        }
        (void)hipFree(dbuf);
        if (hm) (void)hipHostFree(hm);
      } else {
        printf("{\"what\": \"zerocopy\", \"status\": \"setup failed\"}\n");
      }
      if (st) (void)hipStreamDestroy(st);
      (void)hipFree(dh);
      (void)hipFree(dt);
      (void)hipFree(dok);
      (void)hipFree(dm);
      (void)hipHostUnregister(t.img.data());
    }
  }
  // concurrent callers, each with its own table, against the same calls in turn
  if (callers > 1) {
    std::vector<Table> ts(callers);
    for (int c = 0; c < callers; c++) make_table(&ts[c], 100 + c, mib << 20);
    const int per = std::max(1, reps / callers);
    {  // warm: every caller's session exists before either timing
      std::vector<std::thread> w;
      for (int c = 0; c < callers; c++) w.emplace_back([&, c] { (void)seal(ts[c]); });
      for (auto& x : w) x.join();
    }
    const CpuStat a0 = read_cpu_stat();
    double t0 = now();
    bool all_ok = true;
    for (int r = 0; r < per; r++)
      for (int c = 0; c < callers; c++) all_ok = seal(ts[c]).ok() && all_ok;
    const double serial = now() - t0;
    const CpuStat a1 = read_cpu_stat();
    std::atomic<int> fails{0};
    std::vector<std::vector<double>> lat(callers);
    t0 = now();
    std::vector<std::thread> th;
    for (int c = 0; c < callers; c++)
      th.emplace_back([&, c] {
        for (int r = 0; r < per; r++) {
          const double u = now();
          if (!seal(ts[c]).ok()) fails++;
          lat[c].push_back(now() - u);
        }
      });
    for (auto& x : th) x.join();
    const double conc = now() - t0;
    const CpuStat a2 = read_cpu_stat();
    std::vector<double> all;
    for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
    int bad = 0;
    for (auto& tb : ts) bad += check_table(tb);
    printf("{\"what\": \"concurrent_seal\", \"callers\": %d, \"calls_per_caller\": %d, \"bytes_per_call\": %.0f, "
           "\"serial_s\": %.4f, \"serial_GBps\": %.2f, \"concurrent_s\": %.4f, \"concurrent_GBps\": %.2f, "
           "\"speedup\": %.3f, \"concurrent_call_dist\": %s, \"serial_throttled\": %lld, "
           "\"concurrent_throttled\": %lld, \"fails\": %d, \"bad\": %d}\n",
           callers, per, bytes, serial, callers * per * bytes / serial / 1e9, conc,
           callers * per * bytes / conc / 1e9, serial / conc, dist_json(all, bytes).c_str(),
           a1.throttled - a0.throttled, a2.throttled - a1.throttled, fails.load() + (all_ok ? 0 : 1), bad);
  }
  return lsbm_crc32c_shutdown() == LSBM_OK ? 0 : 1;
}
