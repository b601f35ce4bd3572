// tools/db_check_gpu.cc -- every block of every table, and every record of
// every log, of an lsbm database directory checked on the GPU with the
// library's C++ layers only (no reference code linked):
//
//   db_check_gpu DIR [device | --parse-only] [--read=heap] [--filters]
//
// Tables (*.ldb): each file mapped read-only (or, --read=heap, read into a
// writable heap buffer), its footer and index block parsed (the footer of
// table/format.h:50-82 and the block layout of table/block.cc, decoded here),
// and the blocks the reference's verifying reader would check -- the index
// block, every data block it lists, the metaindex block and every block that
// names (the filter) -- gathered as handles.  ONE lsbm::VerifyTables call then
// checks all of them for all tables (ReadBlock's verify, table/format.cc:
// 95-103, batched: mapped images staged through pinned buffers, heap images
// page-locked for the call).  Logs (*.log, MANIFEST-*): lsbm::log::BatchReader,
// one GPU batch per file, then the reference reader's records and Reporter
// calls (common/log_reader.cc:59-162).  --parse-only: the blocks gathered and
// counted, no device call.  --filters: also every table's filter block
// rebuilt on the GPU from its keys and compared byte for byte, and every key
// probed in it (no false negatives).
//
// One JSON line: the counts, every failing block as "file:offset", the
// reporter's calls, and the time of each phase (host CPU too; the device's
// one-time start-up apart).  Checked against tests/cpp/db_verify.cc (the
// reference's own code over the same directory) by tests/test_gpu_parity.py::
// test_db_check_gpu_matches_the_reference_on_a_db_bench_database.
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "lsbm_crc32c.h"
#include "lsbm/filter_block.h"
#include "lsbm/log_checksum.h"
#include "lsbm/table_checksum.h"

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:81
constexpr size_t kFooterSize = 48;                        // 2 handles of <= 20 B + padding + 8 B magic

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double cpu_ms() {
  rusage u;
  getrusage(RUSAGE_SELF, &u);
  return (u.ru_utime.tv_sec + u.ru_stime.tv_sec) * 1e3 + (u.ru_utime.tv_usec + u.ru_stime.tv_usec) * 1e-3;
}

// little-endian varints (util/coding.h's encoding)
bool varint(const char*& p, const char* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint8_t b = static_cast<uint8_t>(*p++);
    r |= static_cast<uint64_t>(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}
uint32_t le32(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

bool handle(const char*& p, const char* end, lsbm::BlockHandle* h) {
  return varint(p, end, &h->offset) && varint(p, end, &h->size);
}

// The entries of block [data, data + n) (contents only, no trailer):
// prefix-compressed entries (key = the previous key's first `shared` bytes +
// the entry's own), then the restart array and its count.  keys (optional)
// receives the full keys, values the values.
bool block_entries(const char* data, size_t n, std::vector<std::string>* keys, std::vector<std::string>* values) {
  if (n < 4) return false;
  const uint32_t restarts = le32(data + n - 4);
  if (restarts > (n - 4) / 4) return false;
  const char* p = data;
  const char* end = data + n - 4 - 4 * (size_t)restarts;
  std::string key;
  while (p < end) {
    uint64_t shared, non_shared, value_len;
    if (!varint(p, end, &shared) || !varint(p, end, &non_shared) || !varint(p, end, &value_len)) return false;
    if ((uint64_t)(end - p) < non_shared + value_len || shared > key.size()) return false;
    key.resize(shared);
    key.append(p, non_shared);
    p += non_shared;
    if (keys) keys->push_back(key);
    if (values) values->emplace_back(p, value_len);
    p += value_len;
  }
  return true;
}
bool block_values(const char* data, size_t n, std::vector<std::string>* values) {
  return block_entries(data, n, nullptr, values);
}

struct Table {
  std::string name;
  std::unique_ptr<char[]> heap;  // --read=heap: the file read into it
  char* bytes = nullptr;         // the image (heap, or a read-only mapping)
  size_t size = 0;
  bool mapped = false;
  std::vector<lsbm::BlockHandle> handles;  // index, data blocks, metaindex, meta blocks
  size_t data_blocks = 0;                  // handles[1, 1 + data_blocks)
  bool has_filter = false;
  lsbm::BlockHandle filter = {0, 0};       // the "filter.<policy>" meta block
  Table() = default;
  Table(Table&& o) noexcept
      : name(std::move(o.name)), heap(std::move(o.heap)), bytes(o.bytes), size(o.size), mapped(o.mapped),
        handles(std::move(o.handles)), data_blocks(o.data_blocks), has_filter(o.has_filter), filter(o.filter) {
    o.bytes = nullptr;
    o.mapped = false;
  }
  ~Table() {
    if (mapped && bytes) munmap(bytes, size);
  }
};

// The blocks of one table: false when it has no footer (a table db_bench was
// still writing when it exited) or its index / metaindex cannot be parsed.
bool table_blocks(Table* t, std::string* why) {
  if (t->size < kFooterSize) return *why = "too short", false;
  const char* f = t->bytes + t->size - kFooterSize;
  uint64_t magic;
  memcpy(&magic, f + kFooterSize - 8, 8);
  if (magic != kTableMagic) return *why = "no footer", false;
  lsbm::BlockHandle meta, index;
  const char* p = f;
  if (!handle(p, f + kFooterSize - 8, &meta) || !handle(p, f + kFooterSize - 8, &index))
    return *why = "bad footer", false;
  auto inside = [&](const lsbm::BlockHandle& h) { return h.offset <= t->size && h.size + 5 <= t->size - h.offset; };
  // (an uncompressed index / metaindex block: db_bench forces kNoCompression,
  // lsbm/db_bench.cc:773; a snappy one would need decoding first)
  auto values = [&](const lsbm::BlockHandle& h, std::vector<std::string>* v) {
    return inside(h) && t->bytes[h.offset + h.size] == lsbm::kNoCompression &&
           block_values(t->bytes + h.offset, h.size, v);
  };
  std::vector<std::string> entries, meta_keys, metas;
  if (!values(index, &entries)) return *why = "index block", false;
  t->handles.push_back(index);
  for (const std::string& e : entries) {
    const char* q = e.data();
    lsbm::BlockHandle h;
    if (!handle(q, e.data() + e.size(), &h)) return *why = "index entry", false;
    t->handles.push_back(h);
  }
  t->data_blocks = entries.size();
  if (!inside(meta) || t->bytes[meta.offset + meta.size] != lsbm::kNoCompression ||
      !block_entries(t->bytes + meta.offset, meta.size, &meta_keys, &metas))
    return *why = "metaindex block", false;
  t->handles.push_back(meta);
  for (size_t i = 0; i < metas.size(); i++) {
    const char* q = metas[i].data();
    lsbm::BlockHandle h;
    if (!handle(q, metas[i].data() + metas[i].size(), &h)) return *why = "metaindex entry", false;
    t->handles.push_back(h);
    if (meta_keys[i].compare(0, 7, "filter.") == 0 && inside(h)) {  // (table/table_builder.cc:280-284)
      t->has_filter = true;
      t->filter = h;
    }
  }
  return true;
}

bool read_file(const std::string& path, std::unique_ptr<char[]>* out, size_t* n) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  out->reset(new char[len > 0 ? len : 1]);
  *n = len > 0 ? (size_t)len : 0;
  const bool ok = fread(out->get(), 1, *n, f) == *n;
  fclose(f);
  return ok;
}

// --read=mmap (the default): the file mapped read-only, its page-cache pages
// mapped in up front (MAP_POPULATE); --read=heap: read into a new buffer
// (the page faults of fresh memory then cost more than the copy: 1.2 GB of
// tables in ~1.1 s here against ~0.07 s mapped)
bool load_table(const std::string& path, bool heap, Table* t) {
  if (heap) {
    if (!read_file(path, &t->heap, &t->size)) return false;
    t->bytes = t->heap.get();
    return true;
  }
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return false;
  }
  t->size = (size_t)st.st_size;
  if (t->size == 0) {
    close(fd);
    static char empty = 0;
    t->bytes = &empty;
    return true;
  }
  void* p = mmap(nullptr, t->size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return false;
  t->bytes = static_cast<char*>(p);
  t->mapped = true;
  return true;
}

struct CountingReporter : public lsbm::log::Reporter {
  uint64_t calls = 0, bytes = 0;
  void Corruption(size_t n, const lsbm::Status&) override {
    calls++;
    bytes += n;
  }
};

std::string json_escape(const std::string& s) {
  std::string r;
  for (char c : s) r += (c == '"' || c == '\\') ? std::string("\\") + c : std::string(1, c);
  return r;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s DIR [device | --parse-only] [--read=heap] [--filters]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const bool parse_only = argc > 2 && strcmp(argv[2], "--parse-only") == 0;
  const int device = argc > 2 && !parse_only ? atoi(argv[2]) : 0;
  bool heap = false, filters = false;
  for (int a = 3; a < argc; a++) {
    heap = heap || strcmp(argv[a], "--read=heap") == 0;
    filters = filters || strcmp(argv[a], "--filters") == 0;
  }
  std::vector<std::string> tables, logs;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      const std::string n = e->d_name;
      if (n.size() > 4 && n.compare(n.size() - 4, 4, ".ldb") == 0) tables.push_back(n);
      else if ((n.size() > 4 && n.compare(n.size() - 4, 4, ".log") == 0) || n.compare(0, 9, "MANIFEST-") == 0)
        logs.push_back(n);
    }
    closedir(d);
  } else {
    fprintf(stderr, "cannot open %s\n", dir.c_str());
    return 1;
  }

  // the device first, timed apart: the HIP runtime's start-up is paid once
  // per process, not per check
  const double ti = now_ms();
  if (!parse_only && lsbm_crc32c_init(device) != 0) {
    fprintf(stderr, "lsbm_crc32c_init(%d) failed\n", device);
    return 1;
  }
  const double t0 = now_ms(), c0 = cpu_ms();
  // the table files read whole by a few threads (they sit in the page cache:
  // the copy and the new buffers' page faults are the cost), then parsed
  std::vector<Table> all(tables.size());
  std::atomic<size_t> next(0);
  std::atomic<bool> read_failed(false);
  const unsigned nthreads = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  std::vector<std::thread> readers;
  for (unsigned w = 0; w < nthreads; w++)
    readers.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < tables.size();) {
        all[i].name = tables[i];
        if (!load_table(dir + "/" + tables[i], heap, &all[i])) read_failed = true;
      }
    });
  for (std::thread& t : readers) t.join();
  if (read_failed) {
    fprintf(stderr, "cannot read a table of %s\n", dir.c_str());
    return 1;
  }
  std::vector<Table> ts;
  std::vector<std::string> unfinished;
  uint64_t bytes = 0;
  for (Table& t : all) {
    std::string why;
    if (!table_blocks(&t, &why)) {
      unfinished.push_back(t.name + " (" + why + ")");
      continue;
    }
    bytes += t.size;
    ts.push_back(std::move(t));
  }
  const double t1 = now_ms();
  std::vector<lsbm::TableImage> images;
  uint64_t blocks = 0;
  for (Table& t : ts) {
    images.push_back(lsbm::TableImage{t.bytes, t.size, t.handles.data(), nullptr, t.handles.size()});
    blocks += t.handles.size();
  }
  std::vector<uint8_t> ok;
  const lsbm::Status vs = parse_only ? lsbm::Status::OK()
                                     : lsbm::VerifyTables(device, images.data(), images.size(), &ok,
                                                          heap ? lsbm::kImagesWritable : lsbm::kImagesReadOnly);
  const double t2 = now_ms();
  // the same call again: the first one of a process also grows the session's
  // pinned staging (a one-time cost, like the device's start-up)
  double again_ms = 0, again_cpu_ms = 0;
  if (!parse_only) {
    const double ac0 = cpu_ms();
    std::vector<uint8_t> ok2;
    const double a0 = now_ms();
    const lsbm::Status s2 = lsbm::VerifyTables(device, images.data(), images.size(), &ok2,
                                               heap ? lsbm::kImagesWritable : lsbm::kImagesReadOnly);
    again_ms = now_ms() - a0;
    again_cpu_ms = cpu_ms() - ac0;
    if (ok2 != ok || s2.ok() != vs.ok()) {
      fprintf(stderr, "VerifyTables: the second call disagrees with the first\n");
      return 1;
    }
  }
  const double t2b = now_ms();
  std::vector<std::string> bad;
  size_t k = 0;
  for (const Table& t : ts)
    for (const lsbm::BlockHandle& h : t.handles)
      if (k < ok.size() && !ok[k++]) bad.push_back(t.name + ":" + std::to_string(h.offset));
  if (!vs.ok() && !vs.IsCorruption()) {
    fprintf(stderr, "VerifyTables: %s\n", vs.ToString().c_str());
    return 1;
  }

  uint64_t records = 0, log_bytes = 0;
  (void)t2b;
  CountingReporter rep;
  for (const std::string& n : logs) {
    if (parse_only) break;
    std::unique_ptr<char[]> img;
    size_t len = 0;
    if (!read_file(dir + "/" + n, &img, &len)) return 1;
    log_bytes += len;
    lsbm::log::BatchReader r(img.get(), len, &rep);
    const lsbm::Status s = r.Verify(device);
    if (!s.ok()) {
      fprintf(stderr, "log %s: %s\n", n.c_str(), s.ToString().c_str());
      return 1;
    }
    std::string rec;
    while (r.ReadRecord(&rec)) records++;
  }
  const double t3 = now_ms(), c3 = cpu_ms();

  // --filters: every table's filter block rebuilt on the GPU from the table's
  // own keys, as its TableBuilder built it -- StartBlock(0), each data
  // block's keys, then StartBlock(the offset after the block and its trailer)
  // (table/table_builder.cc:79-81, 129-131, 143-157) -- one FinishFilterBlocks
  // batch for all tables, compared byte for byte with the table's filter
  // block; then every key looked up in it (FilterBlockReader::KeyMayMatch,
  // table/filter_block.cc:78-109, one batch per table): a filter never says
  // no to a key its table holds.  db_bench's policy: 20 bits per key over user
  // keys (lsbm/db_bench.cc:100, InternalFilterPolicy, lsbm/db_impl.cc:110).
  size_t filters_rebuilt = 0, filters_identical = 0, filter_tables_skipped = 0;
  uint64_t keys_probed = 0, false_negatives = 0;
  double filters_build_ms = 0, filters_feed_ms = 0, filters_finish_ms = 0, filters_probe_ms = 0;
  if (filters && !parse_only) {
    const lsbm::BloomOptions bo;  // (bits_per_key 20, internal keys)
    std::vector<std::unique_ptr<lsbm::FilterBlockBuilder>> builders;
    std::vector<lsbm::FilterBlockBuilder*> ptrs;
    std::vector<const Table*> of;
    struct Probe {
      std::vector<uint64_t> block_offsets, key_offsets{0};
      std::string keys;
      std::vector<uint64_t> block_ends;  // per data block: its keys end here; the offset after it
      std::vector<uint64_t> next_offsets;
    };
    std::vector<Probe> probes;
    const double f0 = now_ms();
    // the tables' keys first (parsing, not timed as filter work)
    for (const Table& t : ts) {
      if (!t.has_filter) continue;
      bool plain = true;
      for (size_t i = 1; i <= t.data_blocks && plain; i++)
        plain = t.bytes[t.handles[i].offset + t.handles[i].size] == lsbm::kNoCompression;
      if (!plain) {
        filter_tables_skipped++;  // (a snappy data block would need decoding first)
        continue;
      }
      Probe pr;
      std::vector<std::string> keys;
      for (size_t i = 1; i <= t.data_blocks; i++) {
        const lsbm::BlockHandle& h = t.handles[i];
        keys.clear();
        if (!block_entries(t.bytes + h.offset, h.size, &keys, nullptr)) {
          fprintf(stderr, "%s: data block at %llu does not parse\n", t.name.c_str(), (unsigned long long)h.offset);
          return 1;
        }
        for (const std::string& k : keys) {
          pr.keys += k;
          pr.key_offsets.push_back(pr.keys.size());
          pr.block_offsets.push_back(h.offset);
        }
        pr.block_ends.push_back(pr.key_offsets.size() - 1);
        pr.next_offsets.push_back(h.offset + h.size + lsbm::kBlockTrailerSize);
      }
      of.push_back(&t);
      probes.push_back(std::move(pr));
    }
    // the filter work: the builders fed as TableBuilder feeds them, then one GPU batch
    const double b0 = now_ms();
    for (const Probe& pr : probes) {
      builders.emplace_back(new lsbm::FilterBlockBuilder(bo));
      lsbm::FilterBlockBuilder* fb = builders.back().get();
      fb->StartBlock(0);
      size_t k = 0;
      for (size_t b = 0; b < pr.block_ends.size(); b++) {
        for (; k < pr.block_ends[b]; k++)
          fb->AddKey(pr.keys.data() + pr.key_offsets[k], pr.key_offsets[k + 1] - pr.key_offsets[k]);
        fb->StartBlock(pr.next_offsets[b]);
      }
      ptrs.push_back(fb);
    }
    filters_feed_ms = now_ms() - b0;
    std::vector<std::string> rebuilt(ptrs.size());
    const double fin0 = now_ms();
    const lsbm::Status fs = lsbm::FinishFilterBlocks(device, ptrs.data(), ptrs.size(), rebuilt.data());
    filters_finish_ms = now_ms() - fin0;
    filters_build_ms = now_ms() - f0;
    if (!fs.ok()) {
      fprintf(stderr, "FinishFilterBlocks: %s\n", fs.ToString().c_str());
      return 1;
    }
    const double p0 = now_ms();
    for (size_t j = 0; j < of.size(); j++) {
      const Table& t = *of[j];
      filters_rebuilt++;
      const char* own = t.bytes + t.filter.offset;
      filters_identical += rebuilt[j].size() == t.filter.size && memcmp(rebuilt[j].data(), own, t.filter.size) == 0;
      lsbm::FilterBlockReader rd(bo, own, t.filter.size);
      std::vector<uint8_t> may;
      const Probe& pr = probes[j];
      const size_t nk = pr.block_offsets.size();
      const lsbm::Status ps = rd.KeyMayMatch(device, pr.block_offsets.data(), pr.keys.data(), pr.key_offsets.data(),
                                             nk, &may);
      if (!ps.ok()) {
        fprintf(stderr, "KeyMayMatch: %s\n", ps.ToString().c_str());
        return 1;
      }
      keys_probed += nk;
      for (size_t i = 0; i < nk; i++) false_negatives += may[i] == 0;
    }
    filters_probe_ms = now_ms() - p0;
  }

  printf("{\"tables\": %zu, \"unfinished\": %zu, \"blocks\": %llu, \"table_bytes\": %llu, \"bad_blocks\": [",
         ts.size(), unfinished.size(), (unsigned long long)blocks, (unsigned long long)bytes);
  for (size_t i = 0; i < bad.size(); i++) printf("%s\"%s\"", i ? ", " : "", json_escape(bad[i]).c_str());
  printf("], \"logs\": %zu, \"log_bytes\": %llu, \"records\": %llu, \"log_corruptions\": %llu, "
         "\"dropped_bytes\": %llu, \"device_init_ms\": %.3f, \"read_parse_ms\": %.3f, \"verify_tables_ms\": %.3f, "
         "\"verify_tables_again_ms\": %.3f, "
         "\"logs_ms\": %.3f, \"total_ms\": %.3f, \"host_cpu_ms\": %.3f, \"read_threads\": %u, "
         "\"unfinished_files\": [",
         logs.size(), (unsigned long long)log_bytes, (unsigned long long)records, (unsigned long long)rep.calls,
         (unsigned long long)rep.bytes, t0 - ti, t1 - t0, t2 - t1, again_ms, t3 - t2b, t3 - t0 - again_ms,
         c3 - c0 - again_cpu_ms, nthreads);
  for (size_t i = 0; i < unfinished.size(); i++) printf("%s\"%s\"", i ? ", " : "", json_escape(unfinished[i]).c_str());
  printf("]");
  if (filters)
    printf(", \"filters_rebuilt\": %zu, \"filters_identical\": %zu, \"filter_tables_skipped\": %zu, "
           "\"keys_probed\": %llu, \"false_negatives\": %llu, \"filters_build_ms\": %.3f, "
           "\"filters_feed_ms\": %.3f, \"filters_finish_ms\": %.3f, \"filters_probe_ms\": %.3f",
           filters_rebuilt, filters_identical, filter_tables_skipped, (unsigned long long)keys_probed,
           (unsigned long long)false_negatives, filters_build_ms, filters_feed_ms, filters_finish_ms,
           filters_probe_ms);
  printf("}\n");
  return 0;
}
