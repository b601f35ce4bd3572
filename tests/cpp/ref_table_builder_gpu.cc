// ref_table_builder_gpu.cc -- TEST DRIVER for integration/gpu_table_builder.h,
// built by oracle/Makefile `gputable` from the reference's own table/, util/
// and common/ objects PLUS its own util/crc32c.cc and util/hash.cc (so the
// unmodified TableBuilder in this binary computes its trailers with the
// reference's own CRC code), this repo's liblsbm_crc32c.so and the HIP
// runtime; run on the GPU box by tests/test_gpu_parity.py.
//
// The key stream is a compaction's output as lsbm writes it: internal keys
// (db_bench's "user%019ld" user keys, lsbm/db_bench.cc:1415, + sequence and
// type, common/dbformat.h) in InternalKeyComparator order with 100-byte
// values, cut into tables the way DoCompactionWork does (Finish once
// FileSize() reaches the target size, lsbm/db_impl.cc:843-892).  Each table is
// built twice from the same entries: by the reference's TableBuilder (CPU
// trailers, block by block) and by GpuTableBuilder (trailers reserved, one
// SealBlocks call per table at Finish).  Checks, per table:
//   * the two files are byte-identical;
//   * the GPU-built file opens with the reference's Table::Open and every
//     entry reads back through ReadBlock with verify_checksums on;
//   * exactly one seal call per table, page-locked in place (one per-call
//     lock per table: lsbm_test_locks_taken).
// Then the read side, per table (integration/gpu_table_reader.h): the
// reference's Table::Open + iteration with verify_checksums (ReadBlock's CRC
// on every data block, as a paranoid compaction reads its inputs) against
// OpenVerifiedTable (the whole file read once, ONE VerifyBlocks call over its
// data blocks, iteration from memory without per-block CRCs): the same
// entries; a flipped data-block byte gives both the same status; a flipped
// filter-block byte neither (the reference never checks it either).
// Configs: 16 MiB tables with a 10-bit bloom filter; lsbm's default 8 MiB
// (config::kTargetFileSize, common/params.cc:20) with no filter; 16 KiB blocks
// with kSnappyCompression requested; a 37-entry table; an empty table.
//
// usage: ref_table_builder_gpu [tables_per_config=3]   (OK ... or FAIL lines)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "common/dbformat.h"
#include "integration/gpu_table_builder.h"
#include "integration/gpu_table_reader.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"
#include "lsbm_crc32c.h"

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

class StringSource : public RandomAccessFile {
 public:
  explicit StringSource(const std::string& s) : s_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result, char* scratch) const {
    if (offset > s_.size()) return Status::IOError("read past end");
    n = std::min(n, (size_t)(s_.size() - offset));
    memcpy(scratch, s_.data() + offset, n);  // (a copy, as pread into the caller's buffer)
    *result = Slice(scratch, n);
    return Status::OK();
  }

 private:
  const std::string& s_;
};

// the compaction's entry stream: ascending user keys, descending sequences
struct Stream {
  uint64_t x, k = 0, seq = 1u << 30;
  explicit Stream(uint64_t seed) : x(seed) {}
  uint64_t next() {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    return x;
  }
  void entry(std::string* key, std::string* value) {
    k += 1 + next() % 7;
    char u[32];
    snprintf(u, sizeof(u), "user%019llu", (unsigned long long)k);
    key->clear();
    AppendInternalKey(key, ParsedInternalKey(Slice(u), seq--, kTypeValue));
    value->resize(100);
    for (size_t i = 0; i < 100; i += 8) {
      uint64_t r = next();
      for (size_t b = 0; b < 8 && i + b < 100; b++, r >>= 8) (*value)[i + b] = (char)(' ' + (r & 0xff) % 95);
    }
  }
};

struct Config {
  const char* name;
  uint64_t target;  // FileSize() at which a table is finished
  int bloom_bits;   // 0: no filter
  size_t block_size;
  CompressionType compression;
  int max_entries;  // -1: until target
};

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int tables_per = argc > 1 ? atoi(argv[1]) : 3;
  if (lsbm_crc32c_init(0) != LSBM_OK) {
    printf("FAIL no device: %s\n", lsbm_crc32c_last_error());
    return 1;
  }
  const Config configs[] = {
      {"16MiB_bloom10", 16u << 20, 10, 4096, kNoCompression, -1},
      {"8MiB_nofilter", 8u << 20, 0, 4096, kNoCompression, -1},
      {"4MiB_16KiB_blocks_snappy_requested", 4u << 20, 10, 16384, kSnappyCompression, -1},
      {"37_entries", 1u << 30, 10, 4096, kNoCompression, 37},
      {"empty", 1u << 30, 10, 4096, kNoCompression, 0},
  };
  const InternalKeyComparator icmp(BytewiseComparator());
  size_t total_tables = 0, total_blocks = 0;
  double t_ref = 0, t_gpu = 0, t_ref_read = 0, t_gpu_read = 0;
  uint64_t total_bytes = 0;
  for (const Config& c : configs) {
    const FilterPolicy* bloom = c.bloom_bits ? NewBloomFilterPolicy(c.bloom_bits) : nullptr;
    InternalFilterPolicy* ifp = bloom ? new InternalFilterPolicy(bloom) : nullptr;
    Options opt;
    opt.comparator = &icmp;  // (as DBImpl sanitises them, lsbm/db_impl.cc:100-120)
    opt.filter_policy = ifp;
    opt.block_size = c.block_size;
    opt.compression = c.compression;
    Stream s(0x5EED0000u + (uint64_t)(&c - configs));
    const int ntab = c.max_entries >= 0 ? 1 : tables_per;
    for (int t = 0; t < ntab; t++) {
      // the table's entries, then the same entries through both builders
      std::vector<std::string> keys, vals;
      std::string k, v;
      uint64_t approx = 0;
      // (more than a table's worth: prefix compression packs entries tighter than their raw size)
      while (c.max_entries >= 0 ? (int)keys.size() < c.max_entries : approx < c.target + c.target / 4) {
        s.entry(&k, &v);
        keys.push_back(k);
        vals.push_back(v);
        approx += k.size() + v.size() + 4;
      }
      StringSink ref_file, gpu_file;
      TableBuilder ref(opt, &ref_file);
      GpuTableBuilder gpu(opt, &gpu_file, 0);
      size_t used = 0;
      double t0 = now();
      for (size_t i = 0; i < keys.size(); i++) {
        ref.Add(keys[i], vals[i]);
        used = i + 1;
        if (ref.FileSize() >= c.target) break;
      }
      EXPECT(c.max_entries >= 0 || ref.FileSize() >= c.target);  // (cut at the target, as compaction)
      const Status rs = ref.Finish();
      const double t1 = now();
      for (size_t i = 0; i < used; i++) {
        gpu.Add(keys[i], vals[i]);
        EXPECT(gpu.FileSize() < c.target || i + 1 == used);  // (the same cut point)
      }
      const long locks0 = lsbm_test_locks_taken();
      const Status gs = gpu.Finish();
      const double t2 = now();
      t_ref += t1 - t0;
      t_gpu += t2 - t1;
      EXPECT(rs.ok());
      EXPECT(gs.ok());
      EXPECT(gpu.SealCalls() == 1);
      EXPECT(lsbm_test_locks_taken() == locks0 + 1);  // (the heap image, DMA-ed in place)
      EXPECT(gpu.NumEntries() == ref.NumEntries() && gpu.FileSize() == ref.FileSize());
      EXPECT(gpu_file.data.size() == ref_file.data.size());
      const bool same = gpu_file.data == ref_file.data;
      EXPECT(same);
      if (!same) {
        size_t i = 0;
        while (i < gpu_file.data.size() && i < ref_file.data.size() && gpu_file.data[i] == ref_file.data[i]) i++;
        printf("FAIL %s table %d: first differing byte %zu of %zu\n", c.name, t, i, ref_file.data.size());
      }
      // read back with the reference's reader, checksums verified on every block
      StringSource src(gpu_file.data);
      Table* table = nullptr;
      const Status os = Table::Open(opt, 1000 + t, &src, gpu_file.data.size(), &table);
      EXPECT(os.ok());
      if (os.ok()) {
        ReadOptions ro;
        ro.verify_checksums = true;
        Iterator* it = table->NewIterator(ro);
        size_t n = 0;
        bool match = true;
        for (it->SeekToFirst(); it->Valid(); it->Next(), n++)
          match = match && n < used && it->key() == Slice(keys[n]) && it->value() == Slice(vals[n]);
        EXPECT(it->status().ok());
        EXPECT(match && n == used);
        delete it;
        delete table;
      }
      // ---- read side: the reference's verified iteration vs one GPU verify per table ----
      const size_t meta_blocks = (ifp ? 1 : 0) + 2;  // filter, metaindex, index
      const size_t n_data = gpu.Blocks() - meta_blocks;
      auto ref_read = [&](const std::string& file, size_t* n, bool* match, Status* st) {
        StringSource rsrc(file);  // (pread-like: every Read copies into ReadBlock's buffer)
        Table* rt = nullptr;
        *st = Table::Open(opt, 2000 + t, &rsrc, file.size(), &rt);
        *n = 0;
        *match = true;
        if (!st->ok()) return;
        ReadOptions ro;
        ro.verify_checksums = true;  // (a paranoid compaction's input iterator, lsbm/version_set.cc:2311)
        Iterator* it = rt->NewIterator(ro);
        for (it->SeekToFirst(); it->Valid(); it->Next(), (*n)++)
          *match = *match && *n < used && it->key() == Slice(keys[*n]) && it->value() == Slice(vals[*n]);
        *st = it->status();
        delete it;
        delete rt;
      };
      auto gpu_read = [&](const std::string& file, size_t* n, bool* match, Status* st, size_t* nblk) {
        StringSource gsrc(file);
        TableImageFile* imf = nullptr;
        Table* gt = nullptr;
        *n = 0;
        *match = true;
        *st = OpenVerifiedTable(opt, 3000 + t, &gsrc, file.size(), 0, &imf, &gt, nblk);
        if (!st->ok()) return;
        Iterator* it = gt->NewIterator(ReadOptions());  // (verified above: no per-block CRC)
        for (it->SeekToFirst(); it->Valid(); it->Next(), (*n)++)
          *match = *match && *n < used && it->key() == Slice(keys[*n]) && it->value() == Slice(vals[*n]);
        *st = it->status();
        delete it;
        delete gt;
        delete imf;
      };
      size_t rn = 0, gn = 0, nblk = 0;
      bool rmatch = false, gmatch = false;
      Status rst, gst;
      const double r0 = now();
      ref_read(ref_file.data, &rn, &rmatch, &rst);
      const double r1 = now();
      gpu_read(ref_file.data, &gn, &gmatch, &gst, &nblk);
      const double r2 = now();
      t_ref_read += r1 - r0;
      t_gpu_read += r2 - r1;
      EXPECT(rst.ok() && rmatch && rn == used);
      EXPECT(gst.ok() && gmatch && gn == used);
      EXPECT(nblk == n_data);
      if (n_data > 1) {
        // a flipped byte in a data block: both report ReadBlock's corruption
        std::string bad = ref_file.data;
        const lsbm::BlockHandle& hb = gpu.Handles()[n_data / 2];
        bad[hb.offset + hb.size / 2] ^= 0x08;
        ref_read(bad, &rn, &rmatch, &rst);
        gpu_read(bad, &gn, &gmatch, &gst, &nblk);
        EXPECT(rst.IsCorruption() && gst.IsCorruption());
        EXPECT(rst.ToString() == gst.ToString());
        EXPECT(gst.ToString() == "Corruption: block checksum mismatch");
      }
      if (ifp && used > 0) {
        // a flipped byte in the filter block: neither checks it (the reference
        // reads filters without verify_checksums, table/table.cc:138-144)
        std::string fb = ref_file.data;
        const lsbm::BlockHandle& hf = gpu.Handles()[n_data];
        if (hf.size > 0) fb[hf.offset] ^= 0x01;
        ref_read(fb, &rn, &rmatch, &rst);
        gpu_read(fb, &gn, &gmatch, &gst, &nblk);
        EXPECT(rst.ok() && gst.ok() && rn == used && gn == used);
      }
      printf("%s table %d: %zu entries, %zu blocks, %zu bytes, identical=%d, reference builder %.1f ms, gpu-sealed "
             "builder %.1f ms; verified read: reference %.1f ms, gpu %.1f ms\n",
             c.name, t, used, gpu.Blocks(), gpu_file.data.size(), (int)same, (t1 - t0) * 1e3, (t2 - t1) * 1e3,
             (r1 - r0) * 1e3, (r2 - r1) * 1e3);
      total_tables++;
      total_blocks += gpu.Blocks();
      total_bytes += gpu_file.data.size();
    }
    delete ifp;
    delete bloom;
  }
  // ---- a device that cannot seal or verify (lsbm_test_fail_host_pipeline:
  // the status a copy, launch or staging error returns): the CPU fallback of
  // integration/gpu_fallback.h, the same file bytes and the same statuses ----
  {
    Options opt;
    opt.comparator = &icmp;
    const FilterPolicy* bloom = NewBloomFilterPolicy(10);
    InternalFilterPolicy ifp(bloom);
    opt.filter_policy = &ifp;
    const uint64_t target = 4u << 20;
    Stream s(0xFA170000u);
    std::vector<std::string> keys, vals;
    std::string k, v;
    for (uint64_t approx = 0; approx < target + target / 4; approx += k.size() + v.size() + 4) {
      s.entry(&k, &v);
      keys.push_back(k);
      vals.push_back(v);
    }
    StringSink ref_file, gpu_file;
    TableBuilder ref(opt, &ref_file);
    GpuTableBuilder gpu(opt, &gpu_file, 0);
    size_t used = 0;
    for (size_t i = 0; i < keys.size() && ref.FileSize() < target; i++, used++) ref.Add(keys[i], vals[i]);
    for (size_t i = 0; i < used; i++) gpu.Add(keys[i], vals[i]);
    EXPECT(ref.Finish().ok());
    const uint64_t seals0 = GpuFallbacks().seals.load();
    EXPECT(lsbm_test_fail_host_pipeline(0) == 0);
    const Status gs = gpu.Finish();
    (void)lsbm_test_fail_host_pipeline(-1);
    EXPECT(gs.ok());  // (round 5: IOError "gpu seal", a sticky bg_error_ in lsbm)
    EXPECT(gpu.HostSeals() == 1 && GpuFallbacks().seals.load() == seals0 + 1);
    EXPECT(gpu.LastGpuError().find("injected fault") != std::string::npos);
    const bool same = gpu_file.data == ref_file.data;
    EXPECT(same);
    // the read side: the reference's verified iteration against
    // OpenVerifiedTable with its device call failing, on the good file and on
    // one with a flipped data-block byte
    auto read = [&](const std::string& file, bool gpu_end, Status* st) -> size_t {
      StringSource src(file);
      TableImageFile* imf = nullptr;
      Table* t = nullptr;
      size_t nblk = 0, n = 0;
      bool match = true;
      ReadOptions ro;
      if (gpu_end) {
        EXPECT(lsbm_test_fail_host_pipeline(0) == 0);
        *st = OpenVerifiedTable(opt, 4000, &src, file.size(), 0, &imf, &t, &nblk);
        (void)lsbm_test_fail_host_pipeline(-1);
      } else {
        *st = Table::Open(opt, 4001, &src, file.size(), &t);
        ro.verify_checksums = true;
      }
      if (!st->ok()) return 0;
      Iterator* it = t->NewIterator(ro);
      for (it->SeekToFirst(); it->Valid(); it->Next(), n++)
        match = match && n < used && it->key() == Slice(keys[n]) && it->value() == Slice(vals[n]);
      *st = it->status();
      if (st->ok()) EXPECT(match);  // (a bad block is skipped: fewer entries, and the status says so)
      delete it;
      delete t;
      delete imf;
      return n;
    };
    const uint64_t ver0 = GpuFallbacks().verifies.load();
    Status rst, gst;
    const size_t rn = read(ref_file.data, false, &rst), gn = read(ref_file.data, true, &gst);
    EXPECT(rst.ok() && gst.ok() && rn == used && gn == used);
    EXPECT(GpuFallbacks().verifies.load() == ver0 + 1);
    std::string bad = ref_file.data;
    const lsbm::BlockHandle& hb = gpu.Handles()[gpu.Blocks() / 3];
    bad[hb.offset + hb.size / 2] ^= 0x10;
    read(bad, false, &rst);
    read(bad, true, &gst);
    EXPECT(GpuFallbacks().verifies.load() == ver0 + 2);
    EXPECT(rst.IsCorruption() && rst.ToString() == gst.ToString());
    EXPECT(gst.ToString() == "Corruption: block checksum mismatch");
    printf("device failure: table of %zu entries, %zu blocks sealed on the CPU after \"%s\", identical=%d; "
           "verified reads on the CPU: %s / %s\n",
           used, gpu.Blocks(), gpu.LastGpuError().c_str(), (int)same, "OK", gst.ToString().c_str());
    delete bloom;
  }
  EXPECT(lsbm_test_locked_ranges() == 0);
  printf("%s tables=%zu blocks=%zu bytes=%llu ref_builder_s=%.3f gpu_builder_s=%.3f ref_verified_read_s=%.3f "
         "gpu_verified_read_s=%.3f\n",
         fails ? "FAILED" : "OK", total_tables, total_blocks, (unsigned long long)total_bytes, t_ref, t_gpu,
         t_ref_read, t_gpu_read);
  (void)lsbm_crc32c_shutdown();
  return fails ? 1 : 0;
}
