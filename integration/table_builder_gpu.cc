// integration/table_builder_gpu.cc -- lsbm's leveldb::TableBuilder
// (include/leveldb/table_builder.h) implemented over GpuTableBuilder: the
// reference's class, constructor, methods and public members, so that lsbm's
// BuildTable (lsbm/builder.cc:36) and DoCompactionWork
// (lsbm/db_impl.cc:838-1060) link against it unchanged in place of
// table/table_builder.o, and every table they write is sealed by ONE
// lsbm::SealBlocks call on the GPU at Finish instead of a CPU crc32c::Value +
// Extend per block (table/table_builder.cc:237-255).
//
// Same file bytes as the reference's TableBuilder for the same options and
// key stream (BlockBuilder, FilterBlockBuilder, the index separators, the
// footer and the 12.5% compression rule all come from the reference's own
// code through GpuTableBuilder); FileSize() counts the reserved trailers, so a
// compaction cuts its output files at the same keys.  What differs is only
// when bytes reach the WritableFile: the whole image at Finish, one Append,
// where the reference appends block by block.  A table is valid only after
// Finish in both (DoCompactionWork syncs and installs it after Finish).
//
// lsbm's pre-caching (table/table_builder.cc:195-230, on when
// runtime::pre_caching, lsbm/db_impl.cc:838) is kept with its exact effect on
// the block cache: a data block whose key span [the table's first key, its
// last key so far] overlaps one of the compaction's cachedRanges is inserted
// under (file number, the pending handle's offset -- which at that point still
// holds the PREVIOUS data block's offset, ~0 for the first block, as in the
// reference), cached_block_number counts it, and the block Finish closes is
// never cached.
//
// Built into oracle/_ref/db_bench_gpu by oracle/Makefile `dbbench_gpu` (the
// reference's own db_bench and DB code, this file, liblsbm_crc32c.so) and run
// on the GPU by tests/test_gpu_parity.py (test_db_bench_gpu_tables).
// LSBM_TABLE_DEVICE picks the HIP device (default 0); LSBM_TABLE_STATS=1
// prints, at exit, how many tables and blocks were sealed on the GPU and the
// time Finish took (the first Finish of a process also opens the device: the
// HIP runtime's start-up, 130-330 ms on the MI355X box, which opening the
// device on a thread at process start did not hide -- db_bench's first flush
// comes ~35-50 ms after start).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>

#include "integration/gpu_table_builder.h"
#include "integration/image_pool.h"
#include "leveldb/cache.h"
#include "leveldb/comparator.h"
#include "leveldb/table_builder.h"
#include "table/block.h"
#include "util/coding.h"

namespace leveldb {

namespace {

int TableDevice() {
  const char* e = getenv("LSBM_TABLE_DEVICE");
  return e && *e ? atoi(e) : 0;
}

// The largest table finished so far in this process: the next builder
// reserves its image once at that size instead of regrowing it (each
// regrowth copies the image so far).  A compaction's outputs are all near its
// MaxOutputFileSize; BuildTable's are one memtable each.
std::atomic<uint64_t> g_size_hint(0);

void DeletePreCachedBlock(const Slice&, void* value) { delete reinterpret_cast<Block*>(value); }

std::atomic<uint64_t> g_tables(0), g_blocks(0), g_bytes(0), g_finish_ns(0), g_finish_max_ns(0);
const std::chrono::steady_clock::time_point g_start = std::chrono::steady_clock::now();
std::atomic<uint64_t> g_first_finish_ns(0);

void PrintStats() {
  fprintf(stderr,
          "lsbm_table_stats: tables_sealed_on_gpu=%llu tables_sealed_on_cpu_after_gpu_error=%llu blocks=%llu "
          "bytes=%llu finish_ms_total=%.3f finish_ms_max=%.3f first_finish_at_ms=%.3f\n",
          (unsigned long long)g_tables.load(), (unsigned long long)GpuFallbacks().seals.load(),
          (unsigned long long)g_blocks.load(),
          (unsigned long long)g_bytes.load(), g_finish_ns.load() * 1e-6, g_finish_max_ns.load() * 1e-6,
          g_first_finish_ns.load() * 1e-6);
}


struct StatsAtExit {
  StatsAtExit() {
    const char* e = getenv("LSBM_TABLE_STATS");
    if (e && *e == '1') atexit(PrintStats);
  }
} g_stats_at_exit;

}  // namespace

struct TableBuilder::Rep {
  Rep(TableBuilder* owner, const Options& opt, WritableFile* f)
      : t(owner),
        options(opt),
        file(f),
        hint(g_size_hint.load(std::memory_order_relaxed)),
        image(ImagePool::Default().Take(GpuTableBuilder::ImageBytesFor(hint))),
        gpu(opt, f, TableDevice(), hint, &image->bytes, &ImagePool::Moving, image) {
    gpu.SetDataBlockObserver(&Rep::Observe, this);
  }
  ~Rep() { ImagePool::Default().Give(image); }  // (pooled and kept page-locked: integration/image_pool.h)

  static void Observe(void* arg, const Slice& contents, bool closing) {
    Rep* r = static_cast<Rep*>(arg);
    if (!closing && r->cache_next) r->PreCache(contents);
  }

  // table/table_builder.cc:195-230: does this block's key span overlap a
  // range of the compaction's cachedRanges (two lists, each walked from its
  // cursor; ranges wholly before the table's first key advance the cursor)?
  void PreCache(const Slice& contents) {
    if (options.block_cache == NULL || t->cachedRanges == NULL) return;
    const Comparator* cmp = options.comparator;
    bool overlap = false;
    for (int w = 0; w < 2 && !overlap; w++) {
      const std::vector<Slice*>& ranges = (*t->cachedRanges)[w];
      for (int i = t->rangeCursor[w]; i < static_cast<int>(ranges.size()); i++) {
        const Slice* range = ranges[i];  // [range[0], range[1]]
        if (cmp->Compare(first_key, range[1]) > 0) {
          t->rangeCursor[w]++;  // passed: no later block of this table reaches it
        } else if (cmp->Compare(last_key, range[0]) >= 0) {
          overlap = true;
          t->cached_block_number++;
          break;
        }
      }
    }
    if (!overlap) return;
    // the pending handle still holds the previous data block's (or the
    // default handle's ~0 offset): the reference's cache key
    const std::vector<lsbm::BlockHandle>& placed = gpu.Handles();
    const uint64_t prev_offset = placed.empty() ? ~static_cast<uint64_t>(0) : placed.back().offset;
    char key[16];
    EncodeFixed64(key, file->getFilenumber());
    EncodeFixed64(key + 8, prev_offset);
    char* copy = new char[contents.size()];
    memcpy(copy, contents.data(), contents.size());
    Block* block = new Block(copy, contents.size(), true);
    Cache::Handle* h = options.block_cache->Insert(Slice(key, sizeof(key)), block, block->size(),
                                                   &DeletePreCachedBlock);
    options.block_cache->Release(h);
  }

  TableBuilder* t;
  Options options;  // (the comparator and block cache of the pre-caching)
  WritableFile* file;
  uint64_t hint;
  PooledImage* image;  // (before gpu: GpuTableBuilder builds into it)
  GpuTableBuilder gpu;
  std::string first_key;  // the table's first key
  std::string last_key;   // the last key added
  bool cache_next = false;  // the Flush being run was asked to pre-cache
};

TableBuilder::TableBuilder(const Options& options, WritableFile* file, bool pre_caching)
    : cachedRanges(NULL), cached_block_number(0), rep_(NULL), pre_caching(pre_caching) {
  rangeCursor[0] = rangeCursor[1] = 0;
  rep_ = new Rep(this, options, file);
}

TableBuilder::~TableBuilder() { delete rep_; }

Status TableBuilder::ChangeOptions(const Options& options) {
  Status s = rep_->gpu.ChangeOptions(options);
  if (s.ok()) rep_->options = options;
  return s;
}

void TableBuilder::Add(const Slice& key, const Slice& value) {
  Rep* r = rep_;
  if (!r->gpu.status().ok()) return;
  if (r->gpu.NumEntries() == 0) r->first_key.assign(key.data(), key.size());
  r->last_key.assign(key.data(), key.size());
  // GpuTableBuilder::Add flushes a full block itself: with this builder's
  // pre-caching flag, as the reference's Add calls Flush(pre_caching) (:137-140)
  r->cache_next = pre_caching;
  r->gpu.Add(key, value);
  r->cache_next = false;
}

void TableBuilder::Flush(bool cache) {
  rep_->cache_next = cache;
  rep_->gpu.Flush();
  rep_->cache_next = false;
}

Status TableBuilder::status() const { return rep_->gpu.status(); }

Status TableBuilder::Finish() {
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t zero = 0;
  g_first_finish_ns.compare_exchange_strong(
      zero, std::chrono::duration_cast<std::chrono::nanoseconds>(t0 - g_start).count());
  const Status s = rep_->gpu.Finish();  // (the seal on the GPU and the file's one Append)
  const uint64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  const uint64_t n = rep_->gpu.FileSize();
  if (s.ok()) {
    if (rep_->gpu.HostSeals() == 0) g_tables++;  // (a CPU-sealed table is counted by GpuFallbacks)
    g_blocks += rep_->gpu.Blocks();
    g_bytes += n;
    g_finish_ns += ns;
    uint64_t m = g_finish_max_ns.load(std::memory_order_relaxed);
    while (ns > m && !g_finish_max_ns.compare_exchange_weak(m, ns, std::memory_order_relaxed)) {
    }
  }
  // remember the size for the next builder's image
  uint64_t prev = g_size_hint.load(std::memory_order_relaxed);
  while (n > prev && !g_size_hint.compare_exchange_weak(prev, n, std::memory_order_relaxed)) {
  }
  return s;
}

void TableBuilder::Abandon() { rep_->gpu.Abandon(); }

uint64_t TableBuilder::NumEntries() const { return rep_->gpu.NumEntries(); }

uint64_t TableBuilder::FileSize() const { return rep_->gpu.FileSize(); }

}  // namespace leveldb
