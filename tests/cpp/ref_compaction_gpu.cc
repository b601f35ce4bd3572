// ref_compaction_gpu.cc -- TEST DRIVER: one compaction end to end, the
// reference's way and with both GPU bindings, built by oracle/Makefile
// `gpucompact` from the reference's own table/, util/ and common/ objects plus
// its own util/crc32c.cc and util/hash.cc; run on the GPU box by
// tests/test_gpu_parity.py.
//
// The shape of DoCompactionWork (lsbm/db_impl.cc:843-892 and its input
// iterator, lsbm/version_set.cc:2300-2330) with paranoid_checks on:
//   inputs   K tables (written here by the reference's TableBuilder), their
//            keys interleaved, each iterated with verify_checksums = true;
//   merge    the reference's MergingIterator over the K inputs
//            (table/merger.cc) under InternalKeyComparator;
//   outputs  TableBuilder, a new table once FileSize() reaches the target.
// The GPU side changes only the two checksum ends: each input is opened with
// OpenVerifiedTable (read once, ONE VerifyBlocks call, iterated from memory
// without per-block CRCs) and each output is a GpuTableBuilder (trailers
// reserved, ONE SealBlocks call at Finish).  Checks: the output files are
// byte-identical, table for table; every input block was verified.  Both
// compactions run three times; the steady-state time (the best of rounds 2-3)
// and the first round's are printed.
//
// Built twice (oracle/Makefile gpucompact): gpu_compaction's CPU side is the
// reference's own util/crc32c.cc (slice-by-4); gpu_compaction_l1's
// (-DLSBM_LEVEL1_CPU) is the same table/ code relinked against the library's
// scalar Extend (Level 1 of INTEGRATION.md: the x86 crc32 instruction).
//
// usage: ref_compaction_gpu [inputs=4] [input_mib=16] [output_mib=16]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>

#include <chrono>
#include <string>
#include <vector>

#include "common/dbformat.h"
#include "integration/gpu_table_builder.h"
#include "integration/gpu_table_reader.h"
#include "integration/image_pool.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"
#include "lsbm_crc32c.h"
#include "table/merger.h"

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

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double cpu_now() {  // this process's CPU time, every thread
  struct rusage ru;
  getrusage(RUSAGE_SELF, &ru);
  return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

class StringSink : public WritableFile {
 public:
  std::string data;
  Status Append(const Slice& s) {
    data.append(s.data(), s.size());
    return Status::OK();
  }
  Status Close() { return Status::OK(); }
  Status Flush() { return Status::OK(); }
  Status Sync() { return Status::OK(); }
};

class StringSource : public RandomAccessFile {  // pread-like: every Read copies
 public:
  explicit StringSource(const std::string& s) : s_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result, char* scratch) const {
    if (offset > s_.size()) return Status::IOError("read past end");
    n = std::min(n, (size_t)(s_.size() - offset));
    memcpy(scratch, s_.data() + offset, n);
    *result = Slice(scratch, n);
    return Status::OK();
  }

 private:
  const std::string& s_;
};

uint64_t xs(uint64_t& x) {
  x ^= x << 13, x ^= x >> 7, x ^= x << 17;
  return x;
}

// A builder for one output table (the GPU builder reserves its image at the
// compaction's target size, as DoCompactionWork knows MaxOutputFileSize).
template <class B>
B* make_builder(const Options& opt, WritableFile* f, uint64_t target);
template <>
TableBuilder* make_builder<TableBuilder>(const Options& opt, WritableFile* f, uint64_t) {
  return new TableBuilder(opt, f);
}
// The GPU ends build into pooled images (integration/image_pool.h: kept
// faulted in and page-locked from table to table) unless LSBM_POOL_IMAGES=0.
bool pool_images() {
  static const bool on = [] {
    const char* e = getenv("LSBM_POOL_IMAGES");
    return !(e && *e == '0');
  }();
  return on;
}
struct PooledGpuTableBuilder {
  PooledImage* image;
  GpuTableBuilder b;
  PooledGpuTableBuilder(const Options& opt, WritableFile* f, uint64_t target)
      : image(ImagePool::Default().Take(GpuTableBuilder::ImageBytesFor(target))),
        b(opt, f, 0, target, &image->bytes, &ImagePool::Moving, image) {}
  ~PooledGpuTableBuilder() { ImagePool::Default().Give(image); }
  void Add(const Slice& k, const Slice& v) { b.Add(k, v); }
  Status Finish() { return b.Finish(); }
  uint64_t FileSize() const { return b.FileSize(); }
};
template <>
GpuTableBuilder* make_builder<GpuTableBuilder>(const Options& opt, WritableFile* f, uint64_t target) {
  return new GpuTableBuilder(opt, f, 0, target);
}
template <>
PooledGpuTableBuilder* make_builder<PooledGpuTableBuilder>(const Options& opt, WritableFile* f, uint64_t target) {
  return new PooledGpuTableBuilder(opt, f, target);
}

// Runs the merge of `children` into tables of about `target` bytes, through
// builder B (TableBuilder or GpuTableBuilder); returns the output files.
template <class B>
std::vector<std::string> merge_into_tables(const Options& opt, Iterator** children, int k, uint64_t target,
                                           Status* st) {
  std::vector<std::string> outs;
  Iterator* merged = NewMergingIterator(opt.comparator, children, k);
  StringSink* sink = nullptr;
  B* b = nullptr;
  auto finish = [&]() {
    if (!b) return;
    Status s = b->Finish();
    if (st->ok()) *st = s;
    delete b;
    b = nullptr;
    outs.push_back(sink->data);
    delete sink;
    sink = nullptr;
  };
  for (merged->SeekToFirst(); merged->Valid(); merged->Next()) {
    if (!b) {
      sink = new StringSink;
      b = make_builder<B>(opt, sink, target);
    }
    b->Add(merged->key(), merged->value());
    if (b->FileSize() >= target) finish();
  }
  finish();
  if (st->ok()) *st = merged->status();
  delete merged;  // (deletes the children)
  return outs;
}

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int K = argc > 1 ? atoi(argv[1]) : 4;
  const uint64_t in_bytes = (argc > 2 ? strtoull(argv[2], nullptr, 10) : 16) << 20;
  const uint64_t out_bytes = (argc > 3 ? strtoull(argv[3], nullptr, 10) : 16) << 20;
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  const InternalKeyComparator icmp(BytewiseComparator());
  const FilterPolicy* bloom = NewBloomFilterPolicy(10);
  InternalFilterPolicy ifp(bloom);
  Options opt;
  opt.comparator = &icmp;
  opt.filter_policy = &ifp;
  opt.block_size = 4096;
  opt.compression = kNoCompression;

  // K input tables: input j holds user keys k with k % K == j (interleaved
  // ranges, as overlapping levels), 100-B values, one sequence number per key
  std::vector<std::string> inputs(K);
  uint64_t x = 0x5EED0007, total_entries = 0;
  for (int j = 0; j < K; j++) {
    StringSink sink;
    TableBuilder tb(opt, &sink);
    std::string key, val(100, ' ');
    for (uint64_t i = 0; tb.FileSize() < in_bytes; i++) {
      char u[32];
      snprintf(u, sizeof(u), "user%019llu", (unsigned long long)(i * K + j));
      key.clear();
      AppendInternalKey(&key, ParsedInternalKey(Slice(u), 1000000000ull - i * K - j, kTypeValue));
      for (size_t b = 0; b < 100; b += 8) {
        uint64_t r = xs(x);
        for (size_t q = 0; q < 8 && b + q < 100; q++, r >>= 8) val[b + q] = (char)(' ' + (r & 0xff) % 95);
      }
      tb.Add(key, val);
      total_entries++;
    }
    EXPECT(tb.Finish().ok());
    inputs[j] = sink.data;
  }

  // Three rounds of both compactions: the first GPU round pays the process's
  // one-time costs (the HIP runtime's first-use event, the session's pinned
  // staging, the device tables' first touch); rounds 2-3 are the steady state
  // of a long-running database.
  std::vector<std::string> ref_out, gpu_out;
  Status rs, gs;
  size_t verified = 0;
  double ref_ms[3] = {0, 0, 0}, gpu_ms[3] = {0, 0, 0}, ref_cpu[3] = {0, 0, 0}, gpu_cpu[3] = {0, 0, 0};
  for (int round = 0; round < 3; round++) {
    // ---- the reference: verified input iterators, TableBuilder outputs ----
    const double t0 = now(), c0 = cpu_now();
    std::vector<StringSource*> srcs;
    std::vector<Table*> rtabs;
    std::vector<Iterator*> rits;
    ReadOptions paranoid;
    paranoid.verify_checksums = true;  // (lsbm/version_set.cc:2311 with paranoid_checks)
    paranoid.fill_cache = false;
    for (int j = 0; j < K; j++) {
      srcs.push_back(new StringSource(inputs[j]));
      Table* t = nullptr;
      EXPECT(Table::Open(opt, 10 + j, srcs.back(), inputs[j].size(), &t).ok());
      rtabs.push_back(t);
      rits.push_back(t->NewIterator(paranoid));
    }
    rs = Status::OK();
    ref_out = merge_into_tables<TableBuilder>(opt, rits.data(), K, out_bytes, &rs);
    ref_ms[round] = (now() - t0) * 1e3;
    ref_cpu[round] = (cpu_now() - c0) * 1e3;
    for (Table* t : rtabs) delete t;
    for (StringSource* s : srcs) delete s;
    srcs.clear();

    // ---- the GPU ends: OpenVerifiedTable inputs, GpuTableBuilder outputs ----
    const double t2 = now(), c2 = cpu_now();
    std::vector<TableImageFile*> imfs(K, nullptr);
    std::vector<Table*> gtabs(K, nullptr);
    std::vector<Iterator*> gits;
    verified = 0;
    for (int j = 0; j < K; j++) {
      srcs.push_back(new StringSource(inputs[j]));
      size_t nb = 0;
      EXPECT(OpenVerifiedTable(opt, 20 + j, srcs.back(), inputs[j].size(), 0, &imfs[j], &gtabs[j], &nb,
                               pool_images() ? &ImagePool::Default() : nullptr).ok());
      verified += nb;
      ReadOptions fast;  // (verified above)
      fast.fill_cache = false;
      gits.push_back(gtabs[j]->NewIterator(fast));
    }
    gs = Status::OK();
    gpu_out = pool_images() ? merge_into_tables<PooledGpuTableBuilder>(opt, gits.data(), K, out_bytes, &gs)
                            : merge_into_tables<GpuTableBuilder>(opt, gits.data(), K, out_bytes, &gs);
    gpu_ms[round] = (now() - t2) * 1e3;
    gpu_cpu[round] = (cpu_now() - c2) * 1e3;
    for (Table* t : gtabs) delete t;
    for (TableImageFile* f : imfs) delete f;
    for (StringSource* s : srcs) delete s;
    EXPECT(ref_out == gpu_out);
  }
  EXPECT(rs.ok() && gs.ok());
  EXPECT(ref_out.size() == gpu_out.size() && !ref_out.empty());
  size_t identical = 0;
  uint64_t out_total = 0;
  for (size_t i = 0; i < ref_out.size() && i < gpu_out.size(); i++) {
    identical += ref_out[i] == gpu_out[i];
    out_total += ref_out[i].size();
  }
  EXPECT(identical == ref_out.size());
  uint64_t in_total = 0;
  for (const auto& s : inputs) in_total += s.size();
  const double ref_steady = std::min(ref_ms[1], ref_ms[2]), gpu_steady = std::min(gpu_ms[1], gpu_ms[2]);
  const double ref_cpu_s = std::min(ref_cpu[1], ref_cpu[2]), gpu_cpu_s = std::min(gpu_cpu[1], gpu_cpu[2]);
#ifdef LSBM_LEVEL1_CPU
  const char* cpu_side = "level1_cpu";  // (the table/ code's crc32c::Extend from liblsbm_crc32c.so)
#else
  const char* cpu_side = "reference";  // (the reference's own util/crc32c.cc)
#endif
  printf("%s cpu_side=%s inputs=%d input_bytes=%llu entries=%llu input_blocks_verified=%zu outputs=%zu identical=%zu "
         "output_bytes=%llu cpu_ms=%.1f gpu_ends_ms=%.1f speedup=%.2f cpu_side_cpu_ms=%.1f gpu_ends_cpu_ms=%.1f "
         "first_round_ms=%.1f/%.1f pooled_images=%d\n",
         fails ? "FAILED" : "OK", cpu_side, K, (unsigned long long)in_total, (unsigned long long)total_entries,
         verified, ref_out.size(), identical, (unsigned long long)out_total, ref_steady, gpu_steady,
         ref_steady / gpu_steady, ref_cpu_s, gpu_cpu_s, ref_ms[0], gpu_ms[0], (int)pool_images());
  delete bloom;
  (void)lsbm_crc32c_shutdown();
  return fails ? 1 : 0;
}
