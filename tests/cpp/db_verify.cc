// tests/cpp/db_verify.cc -- the checker of test_db_bench_gpu_tables: a lsbm
// database directory examined with the REFERENCE's own code only (linked
// against the reference's util/crc32c.cc, never liblsbm_crc32c.so; built by
// oracle/Makefile `dbbench_gpu` as oracle/_ref/db_verify).  TEST
// INFRASTRUCTURE.
//
//   db_verify DIR [--open] [--filters]
//
// Per table file (*.ldb): the footer, then EVERY block read through
// the reference's ReadBlock with verify_checksums (table/format.cc:66-103) --
// the index block, each data block it lists, the metaindex block and the
// filter block it names -- and the entries of every data block counted.
// Per log file (*.log, MANIFEST-*): every record read through the reference's
// log::Reader with checksum = true (common/log_reader.cc:228-242), records
// and reported corruptions counted.  With --open (on a copy: recovery writes),
// the database is opened by the reference's DB::Open with paranoid_checks and
// iterated with verify_checksums; the count of live entries and an FNV-1a
// digest over (key, value) pairs in order identify its content.  With
// --filters, every table's filter block is rebuilt by the reference's own
// FilterBlockBuilder from the table's keys (timed) and compared with its own.
// One JSON line.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <set>
#include <string>
#include <vector>

#include "common/dbformat.h"
#include "common/filename.h"
#include "common/log_reader.h"
#include "leveldb/comparator.h"
#include "leveldb/db.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "lsbm/version_edit.h"
#include "table/block.h"
#include "table/filter_block.h"
#include "table/format.h"

using namespace leveldb;

namespace {

struct Counts {
  uint64_t tables = 0, blocks = 0, entries = 0, table_errors = 0, unfinished = 0;
  uint64_t logs = 0, records = 0, log_errors = 0, dropped_bytes = 0;
  std::string first_error;
  void error(const std::string& where, const Status& s) {
    if (first_error.empty()) first_error = where + ": " + s.ToString();
  }
};

// One block's entries (values kept when asked for, counted into `entries`),
// read through ReadBlock with or without verify_checksums.
Status ReadEntries(RandomAccessFile* f, const BlockHandle& h, bool verify, std::vector<std::string>* values,
                   uint64_t* entries, std::vector<std::string>* keys = nullptr) {
  ReadOptions ro;
  ro.verify_checksums = verify;
  BlockContents c;
  Status s = ReadBlock(f, ro, h, &c);
  if (!s.ok()) return s;
  Block b(c);
  Iterator* it = b.NewIterator(BytewiseComparator());
  for (it->SeekToFirst(); it->Valid(); it->Next()) {
    if (values) values->push_back(it->value().ToString());
    if (keys) keys->push_back(it->key().ToString());
    if (entries) ++*entries;
  }
  s = it->status();
  delete it;
  return s;
}

// --filters: one table's data blocks' keys and its filter block, read ahead
// of the timed rebuild
struct FilterJob {
  std::string name;
  std::vector<std::vector<std::string>> block_keys;
  std::vector<uint64_t> next_offsets;  // after each data block and its trailer
  std::string filter;                  // the table's own filter block
};

// listed: whether any MANIFEST edit added this table.  db_bench exits without
// waiting for its background work, so tables being written at that moment
// (a compaction's outputs, a memtable flush) are left unfinished, and no edit
// names them: a missing footer there marks the file unfinished, not corrupt.
// (The reference's builder leaves the blocks written so far; the GPU builder,
// which writes at Finish, an empty file.)  A listed table must verify.
// Every block the verifying reader would check -- the index block, each data
// block, the metaindex block and the blocks it names (the filter) -- goes
// through ReadBlock with verify_checksums; one that fails with a checksum
// mismatch is listed in `bad` as "file:offset" and the walk goes on (the
// index and metaindex are parsed unverified, as Table::Open reads them).
void VerifyTable(Env* env, const std::string& dir, const std::string& name, bool listed, Counts* n,
                 std::vector<std::string>* bad, std::vector<FilterJob>* jobs) {
  const std::string path = dir + "/" + name;
  uint64_t size = 0;
  RandomAccessFile* f = nullptr;
  Status s = env->GetFileSize(path, &size);
  if (s.ok()) s = env->NewRandomAccessFile(path, &f);
  char buf[Footer::kEncodedLength];
  Slice in;
  Footer footer;
  if (s.ok() && size < Footer::kEncodedLength) s = Status::Corruption("file is too short to be an sstable");
  if (s.ok()) s = f->Read(size - Footer::kEncodedLength, Footer::kEncodedLength, &in, buf);
  if (s.ok()) s = footer.DecodeFrom(&in);
  if (!s.ok() && !listed) {
    n->unfinished++;
    delete f;
    return;
  }
  n->tables++;
  // one block checked: a checksum mismatch is listed, anything else stops the table
  auto check = [&](const BlockHandle& h, std::vector<std::string>* values, uint64_t* entries) {
    Status v = ReadEntries(f, h, true, values, entries);
    n->blocks++;
    if (v.ok()) return true;
    if (v.ToString().find("block checksum mismatch") != std::string::npos) {
      bad->push_back(name + ":" + std::to_string(h.offset()));
      return true;
    }
    s = v;
    return false;
  };
  std::vector<std::string> index, meta, meta_keys;
  FilterJob job;
  job.name = name;
  if (s.ok()) s = ReadEntries(f, footer.index_handle(), false, &index, nullptr);
  if (s.ok() && check(footer.index_handle(), nullptr, nullptr)) {
    for (size_t i = 0; s.ok() && i < index.size(); i++) {
      Slice v(index[i]);
      BlockHandle h;
      s = h.DecodeFrom(&v);
      if (s.ok()) check(h, nullptr, &n->entries);
      if (s.ok() && jobs) {
        job.block_keys.emplace_back();
        s = ReadEntries(f, h, false, nullptr, nullptr, &job.block_keys.back());
        job.next_offsets.push_back(h.offset() + h.size() + kBlockTrailerSize);
      }
    }
  }
  if (s.ok()) s = ReadEntries(f, footer.metaindex_handle(), false, &meta, nullptr, &meta_keys);
  if (s.ok() && check(footer.metaindex_handle(), nullptr, nullptr)) {
    for (size_t i = 0; s.ok() && i < meta.size(); i++) {  // the filter block(s): raw bytes, verified
      Slice v(meta[i]);
      BlockHandle h;
      s = h.DecodeFrom(&v);
      if (!s.ok()) break;
      ReadOptions ro;
      ro.verify_checksums = true;
      BlockContents c;
      Status r = ReadBlock(f, ro, h, &c);
      n->blocks++;
      if (r.ok()) {
        if (jobs && meta_keys[i].compare(0, 7, "filter.") == 0) job.filter.assign(c.data.data(), c.data.size());
        if (c.heap_allocated) delete[] c.data.data();
      } else if (r.ToString().find("block checksum mismatch") != std::string::npos) {
        bad->push_back(name + ":" + std::to_string(h.offset()));
      } else {
        s = r;
      }
    }
  }
  if (!s.ok()) {
    n->table_errors++;
    n->error(path, s);
  } else if (jobs && !job.filter.empty()) {
    jobs->push_back(std::move(job));
  }
  delete f;
}

struct LogReporter : public log::Reader::Reporter {
  Counts* n;
  std::string path;
  void Corruption(size_t bytes, const Status& s) override {
    n->log_errors++;
    n->dropped_bytes += bytes;
    n->error(path, s);
  }
};

void VerifyLog(Env* env, const std::string& path, Counts* n) {
  n->logs++;
  SequentialFile* f = nullptr;
  Status s = env->NewSequentialFile(path, &f);
  if (!s.ok()) {
    n->log_errors++;
    n->error(path, s);
    return;
  }
  LogReporter rep;
  rep.n = n;
  rep.path = path;
  log::Reader reader(f, &rep, true /* checksum */, 0);
  Slice rec;
  std::string scratch;
  while (reader.ReadRecord(&rec, &scratch)) n->records++;
  delete f;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s DIR [--open]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  bool open = false, filters = false;
  for (int a = 2; a < argc; a++) {
    open = open || strcmp(argv[a], "--open") == 0;
    filters = filters || strcmp(argv[a], "--filters") == 0;
  }
  std::vector<FilterJob> jobs;
  Env* env = Env::Default();
  std::vector<std::string> files;
  Status s = env->GetChildren(dir, &files);
  if (!s.ok()) {
    fprintf(stderr, "%s\n", s.ToString().c_str());
    return 1;
  }
  Counts n;
  std::vector<std::string> bad;  // every block that fails its checksum, "file:offset"
  // every table any MANIFEST edit added (lsbm/version_edit.h: four kinds of
  // sorted tables), read with the reference's VersionEdit::DecodeFrom
  std::set<uint64_t> listed;
  for (size_t i = 0; i < files.size(); i++) {
    uint64_t number;
    FileType type;
    if (!ParseFileName(files[i], &number, &type) || type != kDescriptorFile) continue;
    SequentialFile* f = nullptr;
    if (!env->NewSequentialFile(dir + "/" + files[i], &f).ok()) continue;
    Counts ignore;
    LogReporter rep;
    rep.n = &ignore;
    log::Reader reader(f, &rep, true, 0);
    Slice rec;
    std::string scratch;
    while (reader.ReadRecord(&rec, &scratch)) {
      VersionEdit edit;
      if (!edit.DecodeFrom(rec).ok()) continue;
      std::vector<std::pair<int, FileMetaData>>* added = edit.GetNewFiles();
      for (int k = 0; k < 4; k++)
        for (size_t j = 0; j < added[k].size(); j++) listed.insert(added[k][j].second.number);
    }
    delete f;
  }
  for (size_t i = 0; i < files.size(); i++) {
    uint64_t number;
    FileType type;
    if (!ParseFileName(files[i], &number, &type)) continue;
    const std::string path = dir + "/" + files[i];
    if (type == kTableFile)
      VerifyTable(env, dir, files[i], listed.count(number) != 0, &n, &bad, filters ? &jobs : nullptr);
    else if (type == kLogFile || type == kDescriptorFile)
      VerifyLog(env, path, &n);
  }
  // --filters: every table's filter block rebuilt by the reference's own
  // FilterBlockBuilder from the table's keys, fed as TableBuilder feeds it
  // (StartBlock(0), AddKey per key, StartBlock after each data block) with
  // db_bench's policy (InternalFilterPolicy over NewBloomFilterPolicy(20),
  // lsbm/db_bench.cc:100, lsbm/db_impl.cc:110), timed, and compared with the
  // table's own block
  size_t filters_identical = 0;
  double filters_ms = 0;
  if (filters) {
    const FilterPolicy* bloom = NewBloomFilterPolicy(20);
    InternalFilterPolicy ifp(bloom);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::string> rebuilt;
    for (const FilterJob& j : jobs) {
      FilterBlockBuilder fb(&ifp);
      fb.StartBlock(0);
      for (size_t b = 0; b < j.block_keys.size(); b++) {
        for (const std::string& k : j.block_keys[b]) fb.AddKey(k);
        fb.StartBlock(j.next_offsets[b]);
      }
      rebuilt.push_back(fb.Finish().ToString());
    }
    filters_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (size_t i = 0; i < jobs.size(); i++) filters_identical += rebuilt[i] == jobs[i].filter;
    delete bloom;
  }
  uint64_t live = 0, digest = 1469598103934665603ull;  // FNV-1a 64
  std::string open_error;
  if (open) {
    config::db_path = dir.c_str();  // (lsbm's global, set by db_bench's --db, lsbm/db_bench.cc:1802)
    Options o;
    o.paranoid_checks = true;
    DB* db = nullptr;
    s = DB::Open(o, dir, &db);
    if (s.ok()) {
      ReadOptions ro;
      ro.verify_checksums = true;
      Iterator* it = db->NewIterator(ro);
      for (it->SeekToFirst(); it->Valid(); it->Next()) {
        live++;
        const Slice parts[2] = {it->key(), it->value()};
        for (int p = 0; p < 2; p++) {
          const uint64_t len = parts[p].size();
          for (int k = 0; k < 8; k++) digest = (digest ^ ((len >> (8 * k)) & 0xff)) * 1099511628211ull;
          for (size_t k = 0; k < parts[p].size(); k++)
            digest = (digest ^ static_cast<uint8_t>(parts[p][k])) * 1099511628211ull;
        }
      }
      s = it->status();
      delete it;
      delete db;
    }
    if (!s.ok()) open_error = s.ToString();
  }
  printf("{\"tables\": %llu, \"unfinished\": %llu, \"blocks\": %llu, \"entries\": %llu, \"table_errors\": %llu, \"logs\": %llu, "
         "\"records\": %llu, \"log_errors\": %llu, \"dropped_bytes\": %llu, \"first_error\": \"%s\"",
         (unsigned long long)n.tables, (unsigned long long)n.unfinished, (unsigned long long)n.blocks, (unsigned long long)n.entries,
         (unsigned long long)n.table_errors, (unsigned long long)n.logs, (unsigned long long)n.records,
         (unsigned long long)n.log_errors, (unsigned long long)n.dropped_bytes, n.first_error.c_str());
  if (filters)
    printf(", \"filters_rebuilt\": %zu, \"filters_identical\": %zu, \"filters_ms\": %.3f", jobs.size(),
           filters_identical, filters_ms);
  printf(", \"bad_blocks\": [");
  for (size_t i = 0; i < bad.size(); i++) printf("%s\"%s\"", i ? ", " : "", bad[i].c_str());
  printf("]");
  if (open)
    printf(", \"live\": %llu, \"digest\": \"%016llx\", \"open_error\": \"%s\"", (unsigned long long)live,
           (unsigned long long)digest, open_error.c_str());
  printf("}\n");
  return n.table_errors || n.log_errors || !bad.empty() || !open_error.empty() ? 1 : 0;
}
