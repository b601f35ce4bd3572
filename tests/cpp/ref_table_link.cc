// ref_table_link.cc -- TEST DRIVER for tests/test_ref_link.py (build container only).
//
// Drives the reference's OWN, unmodified table/ and common/log_* code through
// its public API: TableBuilder (table/table_builder.cc) writes an SSTable with
// a bloom filter block, log::Writer (common/log_writer.cc) writes a WAL; then
// Table::Open + an iterator with ReadOptions::verify_checksums re-reads every
// block through ReadBlock (table/format.cc:66-148) and log::Reader replays the
// WAL with checksums on.  Finally one byte of a data block is flipped and the
// table is read again: ReadBlock must report "block checksum mismatch".
//
// oracle/Makefile builds this twice from the same reference objects: once
// with the reference's util/crc32c.cc (and util/hash.cc), once with neither,
// linked against lsbm_amd/liblsbm_crc32c.so and compiled with this repo's
// include/ first on the path, so util/crc32c.h and util/hash.h are ours.
// The test compares the two runs' files byte for byte and their output.
//
// usage: ref_table_link <outdir>   (prints one summary line per check)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "common/log_reader.h"
#include "common/log_writer.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"
#include "util/crc32c.h"

using namespace leveldb;

namespace {

std::string value_for(int i) {  // printable, 100 B, like db_bench's values
  std::string v(100, ' ');
  uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
  for (size_t k = 0; k < v.size(); k++) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    v[k] = (char)(' ' + (x >> 40) % 95);
  }
  return v;
}

struct CountingReporter : public log::Reader::Reporter {
  size_t dropped = 0;
  void Corruption(size_t bytes, const Status& s) override {
    dropped += bytes;
    printf("log corruption: %zu bytes: %s\n", bytes, s.ToString().c_str());
  }
};

int read_table(Env* env, const std::string& fname, const Options& opt, int* entries,
               std::string* status) {
  uint64_t size = 0;
  RandomAccessFile* file = nullptr;
  Status s = env->GetFileSize(fname, &size);
  if (s.ok()) s = env->NewRandomAccessFile(fname, &file);
  Table* table = nullptr;
  if (s.ok()) s = Table::Open(opt, 1, file, size, &table);
  *entries = 0;
  if (s.ok()) {
    ReadOptions ro;
    ro.verify_checksums = true;  // every block through ReadBlock's crc check
    Iterator* it = table->NewIterator(ro);
    for (it->SeekToFirst(); it->Valid(); it->Next()) (*entries)++;
    s = it->status();
    delete it;
  }
  *status = s.ToString();
  delete table;
  delete file;
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <outdir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  Env* env = Env::Default();
  Options opt;
  opt.compression = kNoCompression;  // as db_bench (lsbm/db_bench.cc:773)
  opt.filter_policy = NewBloomFilterPolicy(20);
  opt.block_size = 4096;

  // ---- SSTable through TableBuilder::WriteRawBlock ----
  const std::string tname = dir + "/000001.sst";
  WritableFile* wf = nullptr;
  Status s = env->NewWritableFile(tname, &wf);
  if (!s.ok()) return fprintf(stderr, "%s\n", s.ToString().c_str()), 1;
  TableBuilder* tb = new TableBuilder(opt, wf);
  const int kEntries = 20000;
  char key[32];
  for (int i = 0; i < kEntries; i++) {
    snprintf(key, sizeof(key), "user%019d", i);  // lsbm/db_bench.cc:1415
    tb->Add(Slice(key, strlen(key)), value_for(i));
  }
  s = tb->Finish();
  const uint64_t tsize = tb->FileSize();
  delete tb;
  if (s.ok()) s = wf->Close();
  delete wf;
  printf("table: %s size %llu\n", s.ToString().c_str(), (unsigned long long)tsize);

  int entries = 0;
  std::string st;
  read_table(env, tname, opt, &entries, &st);
  printf("table read (verify_checksums): %s entries %d\n", st.c_str(), entries);

  // ---- WAL through log::Writer::EmitPhysicalRecord ----
  const std::string lname = dir + "/000002.log";
  s = env->NewWritableFile(lname, &wf);
  if (!s.ok()) return 1;
  {
    log::Writer w(wf);
    for (int i = 0; i < 3000; i++) {
      const size_t len = (size_t)((i * 7919u) % 40000u);  // spans FIRST/MIDDLE/LAST fragments
      std::string rec(len, 'a');
      for (size_t k = 0; k < len; k++) rec[k] = (char)('a' + (i + k * 31) % 26);
      s = w.AddRecord(rec);
      if (!s.ok()) break;
    }
  }
  if (s.ok()) s = wf->Close();
  delete wf;
  printf("log: %s\n", s.ToString().c_str());
  SequentialFile* sf = nullptr;
  s = env->NewSequentialFile(lname, &sf);
  if (s.ok()) {
    CountingReporter rep;
    log::Reader r(sf, &rep, true /* checksum */, 0);
    Slice rec;
    std::string scratch;
    int n = 0;
    uint32_t h = 0;
    while (r.ReadRecord(&rec, &scratch)) {
      n++;
      h = crc32c::Extend(h, rec.data(), rec.size());
    }
    printf("log read: records %d dropped %zu digest %08x\n", n, rep.dropped, h);
    delete sf;
  }

  // ---- a flipped byte inside the first data block -> ReadBlock corruption ----
  {
    std::string data;
    s = ReadFileToString(env, tname, &data);
    if (s.ok() && data.size() > 100) {
      data[77] ^= 0x20;
      const std::string cname = dir + "/000003.sst";
      s = WriteStringToFile(env, data, cname);
      read_table(env, cname, opt, &entries, &st);
      printf("corrupted table read: %s entries %d\n", st.c_str(), entries);
    }
  }
  printf("scalar: Value(\"123456789\") = %08x Mask = %08x\n", crc32c::Value("123456789", 9),
         crc32c::Mask(crc32c::Value("123456789", 9)));
  delete opt.filter_policy;
  return 0;
}
