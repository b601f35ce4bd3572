// log_checksum.cc -- include/lsbm/log_checksum.h on top of the C ABI.
//
// Writer side: framing on the host (it is a memcpy), every header CRC of a
// batch in one lsbm_log_seal_dev launch.  Reader side: a parallel walk over the
// image's 32 KiB blocks finds every header the reference reader could check, one
// lsbm_log_verify_dev launch checks them all, and a second walk replays
// log::Reader::ReadRecord / ReadPhysicalRecord (common/log_reader.cc:59-256)
// with those results, so records and Reporter calls come out in the
// reference's order.
#include "../../include/lsbm/log_checksum.h"

#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>

#include "../../include/lsbm_crc32c.h"
#include "host_session.h"

namespace lsbm {
namespace log {

namespace {


// The CRC work of a log image through the device's HostSession stages
// (host_session.h), three chunks in flight.  Records [0, n) have their headers
// at heads[] (ascending, inside [lo, hi)); chunks are the image's 4-64 MiB
// windows, and physical records never cross a 32 KiB log block
// (common/log_writer.cc:33-40), so none crosses a window.  seal: res[4i..] =
// the masked crc of record i (lsbm_log_crcs_dev, the image on the device is
// not written); verify: res[i] = its checksum verdict (lsbm_log_verify_dev).
// seal_into (seal only, nullable): instead of res, each chunk's masked crcs
// are stored into the headers at seal_into + heads[i] (EncodeFixed32) as
// soon as the chunk completes, under the later chunks' DMAs.
Status run_log(int device, const char* img, uint64_t lo, uint64_t hi, const uint64_t* heads,
               size_t n, bool seal, uint8_t* res, char* seal_into = nullptr) {
  if (n == 0) return Status::OK();
  HostTiming tm(seal ? "log_seal_device" : "log_verify_device");
  struct Chunk {
    uint64_t lo, hi;
    size_t first, count;
  };
  // windows of a multiple of kBlockSize, so that no record crosses one
  const uint64_t kLogChunk = HostSession::chunk_for(hi - lo) / kBlockSize * kBlockSize;
  // (one search per window: a division per header cost ~10 ms per 1 GB log)
  std::vector<Chunk> chunks;
  for (size_t i = 0; i < n;) {
    const uint64_t w = heads[i] / kLogChunk;
    const size_t j = (size_t)(std::lower_bound(heads + i, heads + n, (w + 1) * kLogChunk) - heads);
    chunks.push_back(Chunk{std::max(lo, w * kLogChunk), std::min(hi, (w + 1) * kLogChunk), i, j - i});
    i = j;
  }
  const bool pinned = host_pinned(img + lo, hi - lo);
  SessionLease s;
  Status st = s.Open(device);
  if (!st.ok()) return st;
  const size_t per = seal ? 4 : 1;
  // the stages' buffers at their largest chunk's size, once: growing them
  // chunk by chunk re-allocates page-locked memory mid-pipeline (a free that
  // waits for the device; ~15 ms per 1 GB group commit)
  size_t max_count = 0;
  for (const Chunk& c : chunks) max_count = std::max(max_count, c.count);
  auto finish = [&](Stage& sg) -> Status {
    double t = tm.on ? HostTiming::now() : 0.0;
    const hipError_t e = s->wait(sg);
    if (tm.on) tm.add(HostTiming::kWait, HostTiming::now() - t), t = HostTiming::now();
    if (e != hipSuccess) return hip_status(e, seal ? "seal" : "verify");
    const Chunk& c = chunks[sg.tag];
    if (seal && seal_into) {
      for (size_t i = 0; i < c.count; i++) {  // [masked crc LE32] at each header (log_writer.cc:85-88)
        uint32_t m;
        memcpy(&m, sg.res.h + 4 * i, 4);
        char* h = seal_into + heads[c.first + i];
        for (int b = 0; b < 4; b++) h[b] = (char)(m >> (8 * b));
      }
    } else {
      memcpy(res + c.first * per, sg.res.h, c.count * per);
    }
    if (tm.on) tm.add(HostTiming::kPost, HostTiming::now() - t);
    return Status::OK();
  };
  for (size_t k = 0; k < chunks.size(); k++) {
    Stage& sg = s->stage((int)(k % HostSession::kStages));
    if (sg.busy) {
      st = finish(sg);
      if (!st.ok()) return st;
    }
    if (host_fault_point(k)) return Status::IOError("injected fault");  // (tests)
    const Chunk& c = chunks[k];
    const uint64_t bytes = c.hi - c.lo;
    hipError_t e = sg.bulk.reserve(kLogChunk);
    if (e == hipSuccess) e = sg.meta.reserve(max_count * sizeof(uint64_t));
    if (e == hipSuccess) e = sg.res.reserve_mapped(max_count * per);  // (the kernel writes the host buffer)
    if (e != hipSuccess) return hip_status(e, "staging buffers");
    double tp = tm.on ? HostTiming::now() : 0.0;
    uint64_t* hh = reinterpret_cast<uint64_t*>(sg.meta.h);
    for (size_t i = 0; i < c.count; i++) hh[i] = heads[c.first + i] - c.lo;
    if (tm.on) tm.add(HostTiming::kPrep, HostTiming::now() - tp);
    sg.settled = false;  // (from here on the stage's stream may hold work)
    if (pinned) {
      e = hipMemcpyAsync(sg.bulk.d, img + c.lo, bytes, hipMemcpyHostToDevice, sg.stream);
    } else {
      const double t = tm.on ? HostTiming::now() : 0.0;
      parallel_copy(sg.bulk.h, img + c.lo, bytes);
      if (tm.on) tm.add(HostTiming::kCopy, HostTiming::now() - t);
      e = hipMemcpyAsync(sg.bulk.d, sg.bulk.h, bytes, hipMemcpyHostToDevice, sg.stream);
    }
    tp = tm.on ? HostTiming::now() : 0.0;
    if (e == hipSuccess)
      e = hipMemcpyAsync(sg.meta.d, sg.meta.h, c.count * sizeof(uint64_t), hipMemcpyHostToDevice,
                         sg.stream);
    if (e != hipSuccess) return hip_status(e, "H2D");
    const uint64_t* d_h = reinterpret_cast<const uint64_t*>(sg.meta.d);
    const int rc = seal ? lsbm_log_crcs_dev(sg.bulk.d, bytes, d_h, c.count,
                                            reinterpret_cast<uint32_t*>(sg.res.d), nullptr, sg.stream)
                        : lsbm_log_verify_dev(sg.bulk.d, bytes, d_h, c.count, sg.res.d, nullptr,
                                              sg.stream);
    if (rc != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
    e = hipEventRecord(sg.done, sg.stream);
    if (tm.on) tm.add(HostTiming::kEnqueue, HostTiming::now() - tp);
    if (e != hipSuccess) return hip_status(e, "event");
    sg.busy = true;
    sg.tag = k;
  }
  for (size_t k = chunks.size() > (size_t)HostSession::kStages ? chunks.size() - HostSession::kStages : 0;
       k < chunks.size(); k++) {
    Stage& sg = s->stage((int)(k % HostSession::kStages));
    if (sg.busy) {
      st = finish(sg);
      if (!st.ok()) return st;
    }
  }
  return Status::OK();
}

inline uint32_t header_length(const uint8_t* h) { return (uint32_t)h[4] | ((uint32_t)h[5] << 8); }

// The headers log::Reader meets in one log block [b, e), every checksum
// assumed good: ReadPhysicalRecord (common/log_reader.cc:179-256) hops from
// header to header until fewer than kHeaderSize bytes are left, a length
// reaches past the block ("bad record length") or a zero-type zero-length
// record (preallocated space) ends the block.  Unknown types and records
// before initial_offset are passed over, not ended at; a checksum mismatch
// would drop the rest of the block, so the replay visits a subset of these.
void block_headers(const uint8_t* f, uint64_t b, uint64_t e, std::vector<uint64_t>* out) {
  while (e - b >= (uint64_t)kHeaderSize) {
    const uint32_t length = header_length(f + b);
    if (kHeaderSize + length > e - b) return;
    if (f[b + 6] == kZeroType && length == 0) return;
    out->push_back(b);
    b += kHeaderSize + length;
  }
}

// log::Reader's values beyond the record types (common/log_reader.h:77-85).
// A type byte of 5 or 6 reads as one of them, exactly as in the reference.
enum : unsigned int { kEof = kMaxRecordType + 1, kBadRecord = kMaxRecordType + 2 };

}  // namespace

// log::Reader over an in-memory file (checksum = true, any initial_offset),
// with the GPU's checksum verdicts for the headers block_headers found.  The reader's buffer_
// is file[buf_begin_, buf_end_) and buf_end_ is its end_of_buffer_offset_.
class Walk {
 public:
  Walk(const uint8_t* file, size_t size, uint64_t initial_offset, Reporter* reporter,
       const std::vector<uint64_t>* checked, const std::vector<uint8_t>* ok)
      : file_(file), size_(size), reporter_(reporter), checked_(checked), ok_(ok),
        initial_offset_(initial_offset) {}

  // log::Reader::ReadRecord (common/log_reader.cc:59-162).
  bool ReadRecord(std::string* record, uint64_t* record_offset) {
    if (last_record_offset_ < initial_offset_) SkipToInitialBlock();
    scratch_.clear();
    record->clear();
    bool in_fragmented_record = false;
    uint64_t prospective_offset = 0;
    while (true) {
      const uint64_t physical_offset = buf_begin_;  // end_of_buffer_offset_ - buffer_.size()
      size_t frag = 0, frag_len = 0;
      const unsigned int type = ReadPhysicalRecord(&frag, &frag_len);
      switch (type) {
        case kFullType:
          if (in_fragmented_record && !scratch_.empty())
            Report(scratch_.size(), "partial record without end(1)");
          record->assign(reinterpret_cast<const char*>(file_) + frag, frag_len);
          *record_offset = last_record_offset_ = physical_offset;
          return true;
        case kFirstType:
          if (in_fragmented_record && !scratch_.empty())
            Report(scratch_.size(), "partial record without end(2)");
          prospective_offset = physical_offset;
          scratch_.assign(reinterpret_cast<const char*>(file_) + frag, frag_len);
          in_fragmented_record = true;
          break;
        case kMiddleType:
          if (!in_fragmented_record)
            Report(frag_len, "missing start of fragmented record(1)");
          else
            scratch_.append(reinterpret_cast<const char*>(file_) + frag, frag_len);
          break;
        case kLastType:
          if (!in_fragmented_record) {
            Report(frag_len, "missing start of fragmented record(2)");
          } else {
            scratch_.append(reinterpret_cast<const char*>(file_) + frag, frag_len);
            record->swap(scratch_);
            *record_offset = last_record_offset_ = prospective_offset;
            return true;
          }
          break;
        case kEof:
          if (in_fragmented_record) {
            Report(scratch_.size(), "partial record without end(3)");
            scratch_.clear();
          }
          return false;
        case kBadRecord:
          if (in_fragmented_record) {
            Report(scratch_.size(), "error in middle of record");
            in_fragmented_record = false;
            scratch_.clear();
          }
          break;
        default: {
          char buf[40];
          snprintf(buf, sizeof(buf), "unknown record type %u", type);
          Report(frag_len + (in_fragmented_record ? scratch_.size() : 0), buf);
          in_fragmented_record = false;
          scratch_.clear();
          break;
        }
      }
    }
  }

  uint64_t LastRecordOffset() const { return last_record_offset_; }

 private:
  // log::Reader::SkipToInitialBlock (common/log_reader.cc:35-57): start at the
  // block holding initial_offset_, or the next one when that offset falls in
  // a block's last 6 bytes (a trailer).  The reference calls it again on
  // every ReadRecord until a record at or past the offset is returned, which
  // only ever happens after the end of the file: the buffer is then empty,
  // eof_ is set and the next read returns kEof again.
  void SkipToInitialBlock() {
    const uint64_t in_block = initial_offset_ % kBlockSize;
    uint64_t block_start = initial_offset_ - in_block;
    if (in_block > (uint64_t)kBlockSize - 6) block_start += kBlockSize;
    if (skipped_) {  // the file is at its end (see above)
      buf_begin_ = buf_end_ = block_start;
      pos_ = size_;
      return;
    }
    skipped_ = true;
    buf_begin_ = buf_end_ = block_start;       // end_of_buffer_offset_ = block_start_location
    pos_ = block_start < size_ ? block_start : size_;  // file_->Skip(block_start_location)
  }

  // log::Reader::ReadPhysicalRecord (common/log_reader.cc:179-256); reads
  // come in kBlockSize pieces from the file position pos_.
  unsigned int ReadPhysicalRecord(size_t* frag, size_t* frag_len) {
    while (true) {
      const size_t avail = buf_end_ - buf_begin_;
      if (avail < (size_t)kHeaderSize) {
        if (!eof_) {  // the rest of this block is a trailer: read the next one
          const size_t got = size_ - pos_ < (size_t)kBlockSize ? size_ - pos_ : (size_t)kBlockSize;
          buf_begin_ = pos_;   // (offsets equal file positions: the skip above keeps them so)
          buf_end_ = pos_ + got;
          pos_ += got;
          if (got < (size_t)kBlockSize) eof_ = true;
          continue;
        }
        if (avail == 0) return kEof;
        buf_begin_ = buf_end_;
        Report(avail, "truncated record at end of file");
        return kEof;
      }
      const uint8_t* header = file_ + buf_begin_;
      const uint32_t length = header_length(header);
      // `unsigned int type = header[6]` with a signed char (common/log_reader.cc:211)
      const unsigned int type = (unsigned int)(int)(signed char)header[6];
      if (kHeaderSize + length > avail) {
        buf_begin_ = buf_end_;
        Report(avail, "bad record length");
        return kBadRecord;
      }
      if (type == kZeroType && length == 0) {  // preallocated region: no report
        buf_begin_ = buf_end_;
        return kBadRecord;
      }
      if (!ChecksumOk(buf_begin_)) {
        // the length may be corrupt too: drop the rest of the block
        buf_begin_ = buf_end_;
        Report(avail, "checksum mismatch");
        return kBadRecord;
      }
      *frag = buf_begin_ + kHeaderSize;
      *frag_len = length;
      buf_begin_ += kHeaderSize + length;
      // a physical record that started before initial_offset_ is skipped
      if (buf_begin_ - kHeaderSize - length < initial_offset_) {
        *frag_len = 0;
        return kBadRecord;
      }
      return type;
    }
  }

  bool ChecksumOk(uint64_t header) {
    // the replay visits a subset of the collected headers, in order
    while (next_ < checked_->size() && (*checked_)[next_] < header) next_++;
    return next_ < checked_->size() && (*checked_)[next_] == header && (*ok_)[next_] != 0;
  }

  // log::Reader::ReportDrop (common/log_reader.cc:171-176): drops that begin
  // before initial_offset_ are not reported (uint64 arithmetic, as there).
  void Report(size_t bytes, const char* reason) {
    if (reporter_ && buf_begin_ - (uint64_t)bytes >= initial_offset_)
      reporter_->Corruption(bytes, Status::Corruption(reason));
  }

  const uint8_t* file_;
  size_t size_;
  Reporter* reporter_;
  const std::vector<uint64_t>* checked_;
  const std::vector<uint8_t>* ok_;
  size_t next_ = 0;
  uint64_t initial_offset_;
  uint64_t buf_begin_ = 0, buf_end_ = 0, pos_ = 0;
  uint64_t last_record_offset_ = 0;
  bool eof_ = false, skipped_ = false;
  std::string scratch_;
};

BatchWriter::BatchWriter() : block_offset_(0), sealed_(0) {}

void BatchWriter::AddRecord(const char* data, size_t n) {
  // common/log_writer.cc:27-73: an empty record still emits one fragment
  bool first = true;
  do {
    if (kBlockSize - block_offset_ < kHeaderSize) {  // no room for a header: pad the block
      dest_.append(kBlockSize - block_offset_, '\0');
      block_offset_ = 0;
    }
    const size_t room = kBlockSize - block_offset_ - kHeaderSize;
    const size_t frag = n < room ? n : room;
    const bool last = frag == n;
    const RecordType type =
        first ? (last ? kFullType : kFirstType) : (last ? kLastType : kMiddleType);
    headers_.push_back(dest_.size());
    // header: CRC left zero for Seal(), then length LE16 and type (:80-84)
    const char header[kHeaderSize] = {0, 0, 0, 0, (char)(frag & 0xff), (char)(frag >> 8),
                                      (char)type};
    dest_.append(header, kHeaderSize);
    dest_.append(data, frag);
    block_offset_ += kHeaderSize + (int)frag;
    data += frag;
    n -= frag;
    first = false;
  } while (n > 0);
}

// BatchReader::Verify's device pass, streamed: the image goes through the
// stages in windows of whole 32 KiB log blocks, and each window's headers are
// found by the same worker job that copies it into staging (2 MiB pieces: the
// walk reads the caller's bytes the copy has just loaded, from cache), so the
// header walk overlaps the previous windows' DMA and kernels instead of
// preceding them all.  Appends every header from `first` on (ascending) to
// *heads and its verdict to *ok.
static Status verify_log_streamed(int device, const char* file, uint64_t size, uint64_t first,
                           std::vector<uint64_t>* heads, std::vector<uint8_t>* ok) {
  HostTiming tm("log_verify_streamed");
  const uint8_t* img = reinterpret_cast<const uint8_t*>(file);
  const uint64_t kWin = HostSession::chunk_for(size - first) / kBlockSize * kBlockSize;
  constexpr uint64_t kPiece = 64ull * kBlockSize;  // 2 MiB
  const bool pinned = host_pinned(file + first, size - first);
  SessionLease s;
  Status st = s.Open(device);
  if (!st.ok()) return st;
  heads->reserve(heads->size() + (size - first) / 512);
  struct Win {
    uint64_t lo;
    size_t first, count;
  };
  std::vector<Win> wins;
  auto finish = [&](Stage& sg) -> Status {
    double t = tm.on ? HostTiming::now() : 0.0;
    const hipError_t e = s->wait(sg);
    if (tm.on) tm.add(HostTiming::kWait, HostTiming::now() - t), t = HostTiming::now();
    if (e != hipSuccess) return hip_status(e, "verify");
    const Win& w = wins[sg.tag];
    memcpy(ok->data() + w.first, sg.res.h, w.count);
    if (tm.on) tm.add(HostTiming::kPost, HostTiming::now() - t);
    return Status::OK();
  };
  std::vector<std::vector<uint64_t>> part((size_t)((kWin + kPiece - 1) / kPiece));
  for (uint64_t lo = first, k = 0; lo < size; lo += kWin, k++) {
    const uint64_t hi = std::min(size, lo + kWin);
    Stage& sg = s->stage((int)(k % HostSession::kStages));
    if (sg.busy) {
      st = finish(sg);
      if (!st.ok()) return st;
    }
    if (host_fault_point(k)) return Status::IOError("injected fault");  // (tests)
    hipError_t e = sg.bulk.reserve(kWin);
    if (e != hipSuccess) return hip_status(e, "staging buffers");
    // copy (unless page-locked) and walk, piece by piece
    const size_t np = (size_t)((hi - lo + kPiece - 1) / kPiece);
    const double t0 = tm.on ? HostTiming::now() : 0.0;
    parallel_for(np, [&](size_t q) {
      const uint64_t p0 = lo + q * kPiece, p1 = std::min(hi, p0 + kPiece);
      if (!pinned) parallel_copy(sg.bulk.h + (p0 - lo), file + p0, p1 - p0);  // (inline: nested)
      part[q].clear();
      for (uint64_t b = p0; b < p1; b += kBlockSize)
        block_headers(img, b, std::min<uint64_t>(p1, b + kBlockSize), &part[q]);
    });
    if (tm.on) tm.add(HostTiming::kCopy, HostTiming::now() - t0);
    const size_t first_h = heads->size();
    for (size_t q = 0; q < np; q++) heads->insert(heads->end(), part[q].begin(), part[q].end());
    const size_t count = heads->size() - first_h;
    ok->resize(heads->size(), 0);
    wins.push_back(Win{lo, first_h, count});
    if (count == 0) continue;  // (nothing to check in this window: no stage work)
    // (sized by the window's actual headers; the session keeps them, so they
    // grow only while a call sees a denser window than any before)
    e = sg.meta.reserve(count * sizeof(uint64_t));
    if (e == hipSuccess) e = sg.res.reserve_mapped(count);
    if (e != hipSuccess) return hip_status(e, "staging buffers");
    uint64_t* hh = reinterpret_cast<uint64_t*>(sg.meta.h);
    for (size_t i = 0; i < count; i++) hh[i] = (*heads)[first_h + i] - lo;
    sg.settled = false;  // (from here on the stage's stream may hold work)
    e = pinned ? hipMemcpyAsync(sg.bulk.d, file + lo, hi - lo, hipMemcpyHostToDevice, sg.stream)
               : hipMemcpyAsync(sg.bulk.d, sg.bulk.h, hi - lo, hipMemcpyHostToDevice, sg.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(sg.meta.d, sg.meta.h, count * sizeof(uint64_t), hipMemcpyHostToDevice, sg.stream);
    if (e != hipSuccess) return hip_status(e, "H2D");
    const int rc = lsbm_log_verify_dev(sg.bulk.d, hi - lo, reinterpret_cast<const uint64_t*>(sg.meta.d),
                                       count, sg.res.d, nullptr, sg.stream);
    if (rc != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
    e = hipEventRecord(sg.done, sg.stream);
    if (e != hipSuccess) return hip_status(e, "event");
    sg.busy = true;
    sg.tag = wins.size() - 1;
  }
  for (int i = 0; i < HostSession::kStages; i++) {  // (oldest first: tags ascend with the stage order)
    Stage* oldest = nullptr;
    for (int j = 0; j < HostSession::kStages; j++) {
      Stage& sg = s->stage(j);
      if (sg.busy && (!oldest || sg.tag < oldest->tag)) oldest = &sg;
    }
    if (!oldest) break;
    st = finish(*oldest);
    if (!st.ok()) return st;
  }
  return Status::OK();
}

Status BatchWriter::Seal(int device) {
  const size_t count = headers_.size() - sealed_;
  if (count == 0) return Status::OK();
  HostTiming tm("BatchWriter::Seal");
  // the unsealed tail of the log: every pending header's masked crc (4 B each
  // come back), EncodeFixed32 into its header (util/coding.cc), chunk by
  // chunk as the chunks complete.  LSBM_LOG_POST_AFTER=1 (A/B): all of them
  // after the last chunk, over the worker pool.
  static const bool post_after = getenv("LSBM_LOG_POST_AFTER") != nullptr;
  if (!post_after) {
    Status s = run_log(device, dest_.data(), headers_[sealed_], dest_.size(), &headers_[sealed_], count, true,
                       nullptr, &dest_[0]);
    if (!s.ok()) return s;
    sealed_ = headers_.size();
    return Status::OK();
  }
  std::unique_ptr<uint32_t[]> masked(new uint32_t[count]);
  Status s = run_log(device, dest_.data(), headers_[sealed_], dest_.size(), &headers_[sealed_],
                     count, true, reinterpret_cast<uint8_t*>(masked.get()));
  if (!s.ok()) return s;
  // EncodeFixed32 into each header; scattered 4-byte stores over the whole
  // image, so split over the worker pool
  constexpr size_t kPiece = 1u << 16;
  char* img = &dest_[0];
  const uint64_t* heads = &headers_[sealed_];
  parallel_for((count + kPiece - 1) / kPiece, [&](size_t k) {
    const size_t i1 = std::min(count, (k + 1) * kPiece);
    for (size_t i = k * kPiece; i < i1; i++) {
      char* h = img + heads[i];
      for (int b = 0; b < 4; b++) h[b] = (char)(masked[i] >> (8 * b));
    }
  });
  sealed_ = headers_.size();
  return Status::OK();
}

BatchReader::BatchReader(const char* file, size_t n, Reporter* reporter, uint64_t initial_offset)
    : file_(file), size_(n), reporter_(reporter), initial_offset_(initial_offset), walk_(nullptr),
      last_record_offset_(0) {}

BatchReader::~BatchReader() { delete walk_; }

Status BatchReader::Verify(int device) {
  const uint8_t* img = reinterpret_cast<const uint8_t*>(file_);
  delete walk_;
  walk_ = nullptr;
  headers_.clear();
  ok_.clear();
  {  // pass 1: every header the reader could check (all checksums assumed good),
    // and its verdict.  Records never cross a block (common/log_writer.cc:33-40)
    // and the reader restarts at every block, so blocks are walked independently,
    // window by window as the image streams to the device: the reader's first
    // block (log::Reader::SkipToInitialBlock, common/log_reader.cc:35-57) to
    // the end of the file.
    const uint64_t in_block = initial_offset_ % kBlockSize;
    uint64_t first = initial_offset_ - in_block;
    if (in_block > (uint64_t)kBlockSize - 6) first += kBlockSize;
    if (first < size_) {
      Status s = verify_log_streamed(device, file_, size_, first, &headers_, &ok_);
      if (!s.ok()) return s;
    }
  }
  // pass 2 (ReadRecord): the reader itself, with the GPU's verdicts
  walk_ = new Walk(img, size_, initial_offset_, reporter_, &headers_, &ok_);
  return Status::OK();
}

bool BatchReader::ReadRecord(std::string* record) {
  if (!walk_) return false;  // Verify() has not succeeded
  return walk_->ReadRecord(record, &last_record_offset_);
}

Status ReadLog(int device, const char* file, size_t n, Reporter* reporter,
               std::vector<std::string>* records, std::vector<uint64_t>* offsets,
               uint64_t initial_offset) {
  if (records) records->clear();
  if (offsets) offsets->clear();
  BatchReader reader(file, n, reporter, initial_offset);
  Status s = reader.Verify(device);
  if (!s.ok()) return s;
  std::string rec;
  while (reader.ReadRecord(&rec)) {
    if (records) records->push_back(rec);
    if (offsets) offsets->push_back(reader.LastRecordOffset());
  }
  return Status::OK();
}

}  // namespace log
}  // namespace lsbm
