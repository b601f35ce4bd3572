// table_checksum.cc -- include/lsbm/table_checksum.h on top of the C ABI.
//
// The blocks of one or many table images are packed into chunks of whole
// blocks (with their trailers) of about equal size, at most 64 MiB, and the
// chunks run through a HostSession's stages (host_session.h), four deep:
// while chunk c's bytes cross PCIe, chunk c-1 is checksummed and chunk c-2's
// results come back.  Only 4 B (seal: the masked trailer crc, dense, written
// into the host image by the host) or 1 B (verify: the ok flag) per block
// return to the host, never the image.
//
// A small job -- one 16 MiB table per call, as TableBuilder::Finish makes
// them (lsbm/db_impl.cc:843-892) -- whose images are page-locked (by the
// caller, or by the seal for the call: CallLocks) skips the chunks: each
// table is one whole-image DMA and one kernel on a stage's stream
// (run_small_locked).  Otherwise one 16 MiB table is four 4 MiB chunks, one
// per stage; a pageable chunk's handles and types travel in its staging
// buffer behind its bytes (one DMA per chunk), a page-locked chunk's bytes
// are DMA-ed from the image on the session's copy stream.
#include "../../include/lsbm/table_checksum.h"

#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <numeric>

#include "../../include/lsbm_crc32c.h"
#include "engine_internal.h"
#include "host_session.h"

namespace lsbm {

std::vector<BlockHandle> LayoutBlocks(const std::vector<uint64_t>& sizes, uint64_t* file_size) {
  std::vector<BlockHandle> h(sizes.size());
  uint64_t off = 0;
  for (size_t i = 0; i < sizes.size(); i++) {
    h[i] = BlockHandle{off, sizes[i]};
    off += sizes[i] + kBlockTrailerSize;
  }
  if (file_size) *file_size = off;
  return h;
}

namespace {

Status check_handles(size_t file_size, const BlockHandle* h, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (h[i].offset > file_size || h[i].size > file_size - h[i].offset ||
        file_size - h[i].offset - h[i].size < kBlockTrailerSize)
      return Status::Corruption("truncated block read");  // table/format.cc:88-91
  return Status::OK();
}

// Bytes [lo, hi) of table t, holding its blocks order[first, first + count).
struct Piece {
  uint32_t t;
  uint64_t lo, hi;
  size_t first, count;
  uint64_t dst;  // offset in the chunk
};
struct Chunk {
  std::vector<Piece> pieces;
  uint64_t bytes = 0;
  size_t blocks = 0;
};

struct Plan {
  std::vector<std::vector<size_t>> order;  // per table: block indices by offset
  std::vector<Chunk> chunks;
  size_t max_blocks = 0;
};

// Whole blocks (and trailers) in offset order, packed into chunks of at most
// HostSession::chunk_for(all bytes) (a larger block gets a chunk of its own),
// closed once they reach an equal share of the bytes: no runt chunk at the
// end (a 1-block fifth chunk cost a kernel launch and a blit per 16 MiB
// table, profiles/r04/one_table_trace/summary_call40.txt).
void make_plan(const TableImage* tables, size_t count, Plan* p) {
  p->order.resize(count);
  size_t total = 0;
  for (size_t t = 0; t < count; t++) total += tables[t].file_size;
  const size_t limit = HostSession::chunk_for(total);
  const size_t target = total / std::max<size_t>(1, (total + limit - 1) / limit);
  // (Unequal chunks for one table per call -- a short first one, or shares
  // doubling from 1/15 of the job -- to shorten the staging copy's lead
  // before the first DMA measured no different: 0.40-0.45 ms per 16 MiB table
  // either way, profiles/r04/check16/, check21/, check22/.)
  Chunk cur;
  auto close = [&]() {
    if (cur.blocks == 0) return;
    p->max_blocks = std::max(p->max_blocks, cur.blocks);
    p->chunks.push_back(std::move(cur));
    cur = Chunk();
  };
  for (size_t t = 0; t < count; t++) {
    const TableImage& tb = tables[t];
    std::vector<size_t>& ord = p->order[t];
    ord.resize(tb.n);
    std::iota(ord.begin(), ord.end(), 0);
    bool sorted = true;
    for (size_t i = 1; i < tb.n && sorted; i++)
      sorted = tb.handles[i].offset >= tb.handles[i - 1].offset;
    if (!sorted)
      std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        return tb.handles[a].offset < tb.handles[b].offset;
      });
    bool open = false;  // cur.pieces.back() is this table's and may grow
    for (size_t k = 0; k < tb.n; k++) {
      const BlockHandle& h = tb.handles[ord[k]];
      const uint64_t end = h.offset + h.size + kBlockTrailerSize;
      if (open) {
        Piece& pc = cur.pieces.back();
        const uint64_t hi = std::max(pc.hi, end);
        if (cur.bytes < target && cur.bytes + (hi - pc.hi) <= limit) {
          cur.bytes += hi - pc.hi;
          pc.hi = hi;
          pc.count++;
          cur.blocks++;
          continue;
        }
        close();
      }
      if (cur.blocks && (cur.bytes >= target || cur.bytes + (end - h.offset) > limit)) close();
      cur.pieces.push_back(Piece{(uint32_t)t, h.offset, end, k, 1, cur.bytes});
      cur.bytes += end - h.offset;
      cur.blocks++;
      open = true;
    }
  }
  close();
}

enum class Op { kSeal, kVerify };

// Page-locked jobs up to this many bytes (LSBM_ZERO_COPY_MAX_MB, default 64;
// 0 = never) take run_small_locked instead of the chunk pipeline.
std::atomic<long> g_zero_copy_mb{-1};  // -1: not read yet
size_t zero_copy_max() {
  long v = g_zero_copy_mb.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("LSBM_ZERO_COPY_MAX_MB");
    v = e ? std::max(0L, atol(e)) : 64;
    long expect = -1;
    if (!g_zero_copy_mb.compare_exchange_strong(expect, v)) v = expect;
  }
  return (size_t)v << 20;
}

// A small page-locked job -- one table per call, as TableBuilder::Finish
// makes them (lsbm/db_impl.cc:843-892): each table is ONE DMA of its whole
// image on a stage's stream and one kernel behind it, its handles and types
// read by the kernel from a mapped page-locked buffer and its results
// written into another (no metadata DMA, no cross-stream events), tables
// spread over the stages, then one wait each.  A 16 MiB table's DMA alone
// takes 0.301 ms (55.7 GB/s), the DMA and the verify kernel 0.334 ms, where
// 4 back-to-back DMAs of its quarters take 0.334 ms alone and the kernel's
// own PCIe reads of the image in place (zero copy) 0.39-0.43 ms
// (profiles/r04/check11/one_table.log: dma_* and zerocopy_* lines).
// LSBM_SMALL_LOCKED=zc (A/B): the kernel reads the image in place through its
// device mapping, the seal storing its trailers there as plain byte stores.
// Returns false, having done nothing, when zero copy is asked for and an
// image has no device mapping.
bool small_locked_zero_copy() {
  static const bool zc = [] {
    const char* e = getenv("LSBM_SMALL_LOCKED");
    return e && strcmp(e, "zc") == 0;
  }();
  return zc;
}

bool run_small_locked(HostSession& hs, const TableImage* tables, size_t count, Op op, std::vector<uint8_t>* ok_out,
                      const std::vector<size_t>& ok_base, size_t* nbad_out, HostTiming& tm, Status* st) {
  const bool zc = small_locked_zero_copy();
  std::vector<const uint8_t*> dev(count, nullptr);
  for (size_t t = 0; t < count && zc; t++) {
    if (tables[t].n == 0) continue;
    // (only memory page-locked for this very device: another device's
    // mapping is not this one's)
    hipPointerAttribute_t attr;
    void* p = nullptr;
    if (hipPointerGetAttributes(&attr, tables[t].file) != hipSuccess || attr.type != hipMemoryTypeHost ||
        attr.device != hs.device() || hipHostGetDevicePointer(&p, tables[t].file, 0) != hipSuccess || !p) {
      (void)hipGetLastError();
      return false;
    }
    dev[t] = static_cast<const uint8_t*>(p);
  }
  size_t nbad = 0;
  auto collect = [&](Stage& sg) -> Status {
    double t0 = tm.on ? HostTiming::now() : 0.0;
    const hipError_t e = hs.wait(sg);
    if (tm.on) tm.add(HostTiming::kWait, HostTiming::now() - t0), t0 = HostTiming::now();
    if (e != hipSuccess) return hip_status(e, op == Op::kSeal ? "seal" : "verify");
    const TableImage& tb = tables[sg.tag];
    if (op == Op::kSeal && zc) {
      // (stored in place by the kernel)
    } else if (op == Op::kSeal) {
      // [type][EncodeFixed32(masked crc)] (table_builder.cc:245-249)
      for (size_t b = 0; b < tb.n; b++) {
        uint32_t m;
        memcpy(&m, sg.res.h + 4 * b, 4);
        char* t = tb.file + tb.handles[b].offset + tb.handles[b].size;
        t[0] = (char)tb.types[b];
        for (int q = 0; q < 4; q++) t[1 + q] = (char)(m >> (8 * q));
      }
    } else {
      for (size_t b = 0; b < tb.n; b++) {
        const uint8_t good = sg.res.h[b];
        nbad += good ? 0 : 1;
        if (ok_out) (*ok_out)[ok_base[sg.tag] + b] = good;
      }
    }
    if (tm.on) tm.add(HostTiming::kPost, HostTiming::now() - t0);
    return Status::OK();
  };
  int k = 0;
  size_t enq = 0;
  for (size_t t = 0; t < count; t++) {
    const TableImage& tb = tables[t];
    if (tb.n == 0) continue;
    Stage& sg = hs.stage(k);
    k = (k + 1) % HostSession::kStages;
    if (sg.busy && !(*st = collect(sg)).ok()) return true;
    if (host_fault_point(enq++)) {  // (tests: a failure with tables in flight)
      *st = Status::IOError("injected fault");
      return true;
    }
    hipError_t e = sg.zmeta.reserve_mapped(tb.n * (sizeof(BlockHandle) + 1) + 16);
    if (e == hipSuccess) e = sg.res.reserve_mapped(tb.n * 4 + 16);
    if (e == hipSuccess && !zc) e = sg.bulk.reserve(tb.file_size + 64);  // (+ the kernel's row slack)
    if (e != hipSuccess) {
      *st = hip_status(e, "staging buffers");
      return true;
    }
    memcpy(sg.zmeta.h, tb.handles, tb.n * sizeof(BlockHandle));
    if (op == Op::kSeal) memcpy(sg.zmeta.h + tb.n * sizeof(BlockHandle), tb.types, tb.n);
    const uint64_t* d_h = reinterpret_cast<const uint64_t*>(sg.zmeta.d);
    const uint8_t* d_ty = sg.zmeta.d + tb.n * sizeof(BlockHandle);
    sg.settled = false;
    const uint8_t* img = dev[t];
    if (!zc) {
      e = hipMemcpyAsync(sg.bulk.d, tb.file, tb.file_size, hipMemcpyHostToDevice, sg.stream);
      if (e != hipSuccess) {
        *st = hip_status(e, "H2D");
        return true;
      }
      img = sg.bulk.d;
    }
    const int rc = op == Op::kVerify ? lsbm_sst_verify_dev(img, tb.file_size, d_h, tb.n, sg.res.d, nullptr, sg.stream)
                   : zc ? sst_seal_in_place(const_cast<uint8_t*>(img), tb.file_size, d_h, d_ty, tb.n, sg.stream)
                        : lsbm_sst_trailer_crcs_dev(img, tb.file_size, d_h, d_ty, tb.n,
                                                    reinterpret_cast<uint32_t*>(sg.res.d), nullptr, sg.stream);
    if (rc != LSBM_OK) {
      *st = Status::IOError(lsbm_crc32c_last_error());
      return true;
    }
    e = hipEventRecord(sg.done, sg.stream);
    if (e != hipSuccess) {
      *st = hip_status(e, "event");
      return true;
    }
    sg.busy = true;
    sg.tag = t;
  }
  for (int i = 0; i < HostSession::kStages; i++) {  // (oldest first)
    Stage& sg = hs.stage((k + i) % HostSession::kStages);
    if (sg.busy && !(*st = collect(sg)).ok()) return true;
  }
  if (nbad_out) *nbad_out = nbad;
  *st = Status::OK();
  return true;
}

// The pipeline.  Seal: trailers written into the host images.  Verify: ok[]
// per block, concatenated over the tables in their block order.
Status run(int device, const TableImage* tables, size_t count, Op op, std::vector<uint8_t>* ok_out,
           size_t* nbad_out, bool writable) {
  HostTiming tm(op == Op::kSeal ? "SealTables" : "VerifyTables");
  Plan plan;
  make_plan(tables, count, &plan);
  if (plan.chunks.empty()) return Status::OK();
  std::vector<size_t> ok_base(count + 1, 0);
  for (size_t t = 0; t < count; t++) ok_base[t + 1] = ok_base[t] + tables[t].n;
  std::vector<uint8_t> pinned(count);
  for (size_t t = 0; t < count; t++) pinned[t] = host_pinned(tables[t].file, tables[t].file_size);

  CallLocks locks;  // (before the lease: unlocked after its streams are synchronised)
  SessionLease s;
  Status st = s.Open(device);
  if (!st.ok()) return st;
  {
    size_t total = 0;
    for (size_t t = 0; t < count; t++) total += tables[t].file_size;
    // A small job's pageable images are page-locked for the call and DMA-ed
    // in place: one 16 MiB table per call 0.355 ms, registration included,
    // against 0.39-0.60 ms through the staging copy, box to box
    // (profiles/r04/check17/, seal_register_per_call vs seal_pageable).
    // Big jobs keep the staging pipeline (53.8 against 51.3 GB/s in place,
    // profiles/r04/check13/host_*.log).
    // Verify too, for writable images (lsbm's ReadBlock buffers are heap
    // memory, table/format.cc:79-82): 0.35 ms and ~0.4 ms of host CPU per
    // 16 MiB table against 0.41 ms and ~5 ms through round 4's staging
    // (DESIGN section 5).
    // (not for zero copy: its seal stores into the image, and a read-only
    // registration must never be written by the device)
    if (total <= zero_copy_max() && CallLocks::enabled() && !small_locked_zero_copy())
      for (size_t t = 0; t < count; t++)
        if (!pinned[t] && tables[t].n != 0)
          pinned[t] = locks.add(device, tables[t].file, tables[t].file_size, writable);
    bool all_pinned = true;
    for (size_t t = 0; t < count; t++) all_pinned = all_pinned && (tables[t].n == 0 || pinned[t]);
    if (all_pinned && total <= zero_copy_max() &&
        run_small_locked(*s, tables, count, op, ok_out, ok_base, nbad_out, tm, &st))
      return st;  // (false: zero copy asked for and an image without a device mapping)
  }
  const size_t meta_bytes = plan.max_blocks * (sizeof(BlockHandle) + 1) + 16;
  const size_t res_bytes = plan.max_blocks * 4 + 16;
  // a pageable chunk's staging: its bytes, then (16-B aligned) its handles and types
  size_t max_chunk = 0;
  for (const Chunk& ch : plan.chunks) max_chunk = std::max<size_t>(max_chunk, ch.bytes);
  const size_t bulk_bytes = max_chunk + meta_bytes + 32;
  size_t nbad = 0;

  // chunk sg.tag's results, from its stage (host side)
  auto finish = [&](Stage& sg) -> Status {
    double t = tm.on ? HostTiming::now() : 0.0;
    const hipError_t e = s->wait(sg);
    if (tm.on) tm.add(HostTiming::kWait, HostTiming::now() - t), t = HostTiming::now();
    if (e != hipSuccess) return hip_status(e, op == Op::kSeal ? "seal" : "verify");
    struct Post {
      HostTiming& tm;
      double t;
      ~Post() {
        if (tm.on) tm.add(HostTiming::kPost, HostTiming::now() - t);
      }
    } post{tm, t};
    const Chunk& ch = plan.chunks[sg.tag];
    if (op == Op::kSeal) {
      // [type][EncodeFixed32(masked crc)] (table_builder.cc:245-249): scattered
      // 5-byte stores into the caller's images (each its own page for 4 KiB
      // blocks: a TLB miss and a line fill per trailer), split over the worker
      // pool in runs of kRun blocks: ~0.15 ms per 64 MiB chunk on one thread.
      // A one-table chunk (~1,000 blocks) is one run, on this thread: 256-block
      // runs over the pool took 0.10-0.14 ms per 16 MiB table against ~0.05 ms
      // inline (profiles/r04/check5/timing.log).  The drain below posts each
      // chunk as soon as its stage completes, under the later chunks' DMA.
      constexpr size_t kRun = 2048;
      struct Run {
        const Piece* pc;
        size_t k0, k1, j0;
      };
      std::vector<Run> runs;
      size_t j = 0;
      for (const Piece& pc : ch.pieces) {
        for (size_t k = pc.first; k < pc.first + pc.count; k += kRun)
          runs.push_back(Run{&pc, k, std::min(pc.first + pc.count, k + kRun), j + (k - pc.first)});
        j += pc.count;
      }
      parallel_for(runs.size(), [&](size_t r) {
        const Run& rn = runs[r];
        const TableImage& tb = tables[rn.pc->t];
        for (size_t k = rn.k0, jj = rn.j0; k < rn.k1; k++, jj++) {
          const size_t b = plan.order[rn.pc->t][k];
          uint32_t m;
          memcpy(&m, sg.res.h + 4 * jj, 4);
          char* t = tb.file + tb.handles[b].offset + tb.handles[b].size;
          t[0] = (char)tb.types[b];
          for (int q = 0; q < 4; q++) t[1 + q] = (char)(m >> (8 * q));
        }
      });
      return Status::OK();
    }
    size_t j = 0;
    for (const Piece& pc : ch.pieces) {
      for (size_t k = pc.first; k < pc.first + pc.count; k++, j++) {
        const size_t b = plan.order[pc.t][k];
        const uint8_t good = sg.res.h[j];
        if (!good) nbad++;
        if (ok_out) (*ok_out)[ok_base[pc.t] + b] = good;
      }
    }
    return Status::OK();
  };

  for (size_t c = 0; c < plan.chunks.size(); c++) {
    Stage& sg = s->stage((int)(c % HostSession::kStages));
    if (sg.busy) {
      st = finish(sg);
      if (!st.ok()) return st;
    }
    if (host_fault_point(c)) return Status::IOError("injected fault");  // (tests)
    const Chunk& ch = plan.chunks[c];
    bool direct = true;
    for (const Piece& pc : ch.pieces) direct = direct && pinned[pc.t];
    hipError_t e = sg.bulk.reserve(bulk_bytes);
    if (e == hipSuccess && direct) e = sg.meta.reserve(meta_bytes);
    if (e == hipSuccess) e = sg.res.reserve_mapped(res_bytes);  // (the kernel writes the host buffer)
    if (e != hipSuccess) return hip_status(e, "staging buffers");
    // per-block inputs: handles rebased into the chunk, then the types
    const size_t meta_off = direct ? 0 : (ch.bytes + 15) / 16 * 16;
    uint8_t* meta_h = direct ? sg.meta.h : sg.bulk.h + meta_off;
    uint8_t* meta_d = direct ? sg.meta.d : sg.bulk.d + meta_off;
    BlockHandle* hh = reinterpret_cast<BlockHandle*>(meta_h);
    uint8_t* ty = meta_h + ch.blocks * sizeof(BlockHandle);
    size_t j = 0;
    for (const Piece& pc : ch.pieces) {
      const TableImage& tb = tables[pc.t];
      const std::vector<size_t>& ord = plan.order[pc.t];
      for (size_t k = pc.first; k < pc.first + pc.count; k++, j++) {
        const size_t b = ord[k];
        hh[j] = BlockHandle{tb.handles[b].offset - pc.lo + pc.dst, tb.handles[b].size};
        if (op == Op::kSeal) ty[j] = tb.types[b];
      }
    }
    const size_t meta_n = ch.blocks * sizeof(BlockHandle) + (op == Op::kSeal ? ch.blocks : 0);
    sg.settled = false;  // (from here on the stage's stream may hold work)
    if (direct) {
      // page-locked: the metadata first, then the bytes DMA-ed in place, on
      // the stage's own stream (the stages' DMAs run side by side, as the
      // staged path's do: a 1000-table compaction's verify 53.6 against
      // 51.7 GB/s, seal 50.0-51.2 against 51.7, profiles/r04/check20/; one
      // table per call takes run_small_locked).  LSBM_DIRECT_COPY_STREAM=1
      // (A/B): on the session's copy stream, back to back, the stage's
      // kernel waiting for its chunk.
      static const bool copy_stream = getenv("LSBM_DIRECT_COPY_STREAM") != nullptr;
      hipStream_t cs = sg.stream;
      if (copy_stream) e = s->copy_stream(&cs);
      if (e == hipSuccess) e = hipMemcpyAsync(sg.meta.d, sg.meta.h, meta_n, hipMemcpyHostToDevice, cs);
      for (const Piece& pc : ch.pieces)
        if (e == hipSuccess)
          e = hipMemcpyAsync(sg.bulk.d + pc.dst, tables[pc.t].file + pc.lo, pc.hi - pc.lo,
                             hipMemcpyHostToDevice, cs);
      if (copy_stream && e == hipSuccess) e = hipEventRecord(sg.copied, cs);
      if (copy_stream && e == hipSuccess) e = hipStreamWaitEvent(sg.stream, sg.copied, 0);
    } else {
      // pageable: bytes and metadata through the pinned staging, one DMA
      const double t = tm.on ? HostTiming::now() : 0.0;
      for (const Piece& pc : ch.pieces)
        parallel_copy(sg.bulk.h + pc.dst, tables[pc.t].file + pc.lo, pc.hi - pc.lo);
      if (tm.on) tm.add(HostTiming::kCopy, HostTiming::now() - t);
      e = hipMemcpyAsync(sg.bulk.d, sg.bulk.h, meta_off + meta_n, hipMemcpyHostToDevice, sg.stream);
    }
    if (e != hipSuccess) return hip_status(e, "H2D");
    const uint64_t* d_h = reinterpret_cast<const uint64_t*>(meta_d);
    int rc;
    if (op == Op::kSeal)
      rc = lsbm_sst_trailer_crcs_dev(sg.bulk.d, ch.bytes, d_h, meta_d + ch.blocks * sizeof(BlockHandle),
                                     ch.blocks, reinterpret_cast<uint32_t*>(sg.res.d), nullptr, sg.stream);
    else
      rc = lsbm_sst_verify_dev(sg.bulk.d, ch.bytes, d_h, ch.blocks, sg.res.d, nullptr, sg.stream);
    if (rc != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
    e = hipEventRecord(sg.done, sg.stream);
    if (e != hipSuccess) return hip_status(e, "event");
    sg.busy = true;
    sg.tag = c;
  }
  // the remaining stages, oldest chunk first
  for (size_t c = plan.chunks.size() > (size_t)HostSession::kStages
                      ? plan.chunks.size() - HostSession::kStages : 0;
       c < plan.chunks.size(); c++) {
    Stage& sg = s->stage((int)(c % HostSession::kStages));
    if (sg.busy) {
      st = finish(sg);
      if (!st.ok()) return st;
    }
  }
  if (nbad_out) *nbad_out = nbad;
  return Status::OK();
}

}  // namespace

Status SealTables(int device, const TableImage* tables, size_t count) {
  for (size_t t = 0; t < count; t++) {
    const TableImage& tb = tables[t];
    if (tb.n == 0) continue;
    if (!tb.file || !tb.handles || !tb.types) return Status::InvalidArgument("null pointer");
    Status s = check_handles(tb.file_size, tb.handles, tb.n);
    if (!s.ok()) return s;
  }
  return run(device, tables, count, Op::kSeal, nullptr, nullptr, true);
}

Status VerifyTables(int device, const TableImage* tables, size_t count, std::vector<uint8_t>* ok,
                    ImageMemory memory) {
  size_t total = 0;
  for (size_t t = 0; t < count; t++) total += tables[t].n;
  if (ok) ok->assign(total, 1);
  for (size_t t = 0; t < count; t++) {
    const TableImage& tb = tables[t];
    if (tb.n == 0) continue;
    if (!tb.file || !tb.handles) return Status::InvalidArgument("null pointer");
    Status s = check_handles(tb.file_size, tb.handles, tb.n);
    if (!s.ok()) return s;
  }
  size_t nbad = 0;
  Status s = run(device, tables, count, Op::kVerify, ok, &nbad, memory == kImagesWritable);
  if (!s.ok()) return s;
  return nbad ? Status::Corruption("block checksum mismatch") : Status::OK();
}

Status VerifyTables(int device, const TableImage* tables, size_t count, std::vector<uint8_t>* ok) {
  return VerifyTables(device, tables, count, ok, kImagesReadOnly);
}

Status SealBlocks(int device, char* file, size_t file_size, const BlockHandle* handles,
                  const uint8_t* types, size_t n) {
  if (n == 0) return Status::OK();
  if (!file || !handles || !types) return Status::InvalidArgument("null pointer");
  const TableImage t{file, file_size, handles, types, n};
  return SealTables(device, &t, 1);
}

namespace {
Status verify_one(int device, char* file, size_t file_size, const BlockHandle* handles, size_t n,
                  std::vector<uint8_t>* ok, ImageMemory memory) {
  if (ok) ok->assign(n, 1);
  if (n == 0) return Status::OK();
  if (!file || !handles) return Status::InvalidArgument("null pointer");
  const TableImage t{file, file_size, handles, nullptr, n};
  return VerifyTables(device, &t, 1, ok, memory);
}
}  // namespace

Status VerifyBlocks(int device, const char* file, size_t file_size, const BlockHandle* handles,
                    size_t n, std::vector<uint8_t>* ok, ImageMemory memory) {
  return verify_one(device, const_cast<char*>(file), file_size, handles, n, ok, memory);
}

}  // namespace lsbm

// Testing (include/lsbm_crc32c.h): the zero-copy threshold in MiB (0: never).
extern "C" __attribute__((visibility("default"))) int lsbm_test_zero_copy_max_mb(int mb) {
  if (mb < 0) return -1;
  lsbm::g_zero_copy_mb.store(mb);
  return 0;
}
