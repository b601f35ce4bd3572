// log_checksum.cc -- include/lsbm/log_checksum.h on top of the C ABI.
//
// Writer side: framing on the host (it is a memcpy), every header CRC of a
// batch in one lsbm_log_seal_dev launch.  Reader side: a first walk over the
// image finds every header the reference reader could check, one
// lsbm_log_verify_dev launch checks them all, and a second walk replays
// log::Reader::ReadRecord / ReadPhysicalRecord (common/log_reader.cc:59-256)
// with those results, so records and Reporter calls come out in the
// reference's order.
#include "../../include/lsbm/log_checksum.h"

#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>

#include "../../include/lsbm_crc32c.h"
#include "host_stage.h"

namespace lsbm {
namespace log {

namespace {

Status hip_status(hipError_t e, const char* what) {
  return Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceLog {
  uint8_t* image = nullptr;
  uint64_t* headers = nullptr;
  void* aux = nullptr;  // masked CRCs (seal) or ok flags (verify)
  uint32_t* nbad = nullptr;
  PinnedBounce bounce;
  CallStream stream;
  ~DeviceLog() {
    if (stream.status() == hipSuccess) (void)hipStreamSynchronize(stream.get());
    if (image) (void)hipFree(image);
    if (headers) (void)hipFree(headers);
    if (aux) (void)hipFree(aux);
    if (nbad) (void)hipFree(nbad);
  }
};

// Stage image[0, n) and the header offsets on `device` (host_stage.h).
Status stage(int device, const char* image, size_t n, const uint64_t* headers, size_t count,
             size_t aux_bytes, DeviceLog* d) {
  if (lsbm_crc32c_init(device) != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = d->stream.status();
  if (e == hipSuccess) e = hipMalloc(&d->image, n ? n : 1);
  if (e == hipSuccess) e = hipMalloc(&d->headers, count * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&d->aux, aux_bytes);
  if (e == hipSuccess) e = hipMalloc(&d->nbad, sizeof(uint32_t));
  if (e == hipSuccess) e = d->bounce.to_device(d->image, image, n, d->stream.get());
  if (e == hipSuccess)
    e = d->bounce.to_device(d->headers, headers, count * sizeof(uint64_t), d->stream.get());
  if (e == hipSuccess) e = hipMemsetAsync(d->nbad, 0, sizeof(uint32_t), d->stream.get());
  return e == hipSuccess ? Status::OK() : hip_status(e, "staging");
}

inline uint32_t header_length(const uint8_t* h) { return (uint32_t)h[4] | ((uint32_t)h[5] << 8); }

// log::Reader's values beyond the record types (common/log_reader.h:77-85).
// A type byte of 5 or 6 reads as one of them, exactly as in the reference.
enum : unsigned int { kEof = kMaxRecordType + 1, kBadRecord = kMaxRecordType + 2 };

}  // namespace

// One pass of log::Reader over an in-memory file (checksum = true, any
// initial_offset).  In the collecting pass every header whose checksum the
// reader would test is recorded and assumed good; in the replay pass the
// GPU's verdicts are used and Reporter calls are made.  The reader's buffer_
// is file[buf_begin_, buf_end_) and buf_end_ is its end_of_buffer_offset_.
class Walk {
 public:
  Walk(const uint8_t* file, size_t size, uint64_t initial_offset, Reporter* reporter,
       std::vector<uint64_t>* collect, const std::vector<uint64_t>* checked,
       const std::vector<uint8_t>* ok)
      : file_(file), size_(size), reporter_(reporter), collect_(collect), checked_(checked),
        ok_(ok), initial_offset_(initial_offset) {}

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
    if (collect_) {
      collect_->push_back(header);
      return true;
    }
    // the replay visits a subset of the collected headers, in order
    while (next_ < checked_->size() && (*checked_)[next_] < header) next_++;
    return next_ < checked_->size() && (*checked_)[next_] == header && (*ok_)[next_] != 0;
  }

  // log::Reader::ReportDrop (common/log_reader.cc:171-176): drops that begin
  // before initial_offset_ are not reported (uint64 arithmetic, as there).
  void Report(size_t bytes, const char* reason) {
    if (reporter_ && !collect_ && buf_begin_ - (uint64_t)bytes >= initial_offset_)
      reporter_->Corruption(bytes, Status::Corruption(reason));
  }

  const uint8_t* file_;
  size_t size_;
  Reporter* reporter_;
  std::vector<uint64_t>* collect_;
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

Status BatchWriter::Seal(int device) {
  const size_t count = headers_.size() - sealed_;
  if (count == 0) return Status::OK();
  // stage only the unsealed tail of the log, headers rebased to it
  const uint64_t base = headers_[sealed_];
  std::vector<uint64_t> rebased(count);
  for (size_t i = 0; i < count; i++) rebased[i] = headers_[sealed_ + i] - base;
  DeviceLog d;
  Status s = stage(device, dest_.data() + base, dest_.size() - base, rebased.data(), count,
                   count * sizeof(uint32_t), &d);
  if (!s.ok()) return s;
  if (lsbm_log_seal_dev(d.image, dest_.size() - base, d.headers, count,
                        static_cast<uint32_t*>(d.aux), d.nbad, d.stream.get()) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  std::vector<uint32_t> masked(count);
  uint32_t nbad = 0;
  hipError_t e = d.bounce.to_host(masked.data(), d.aux, count * sizeof(uint32_t), d.stream.get());
  if (e == hipSuccess) e = d.bounce.to_host(&nbad, d.nbad, sizeof(nbad), d.stream.get());
  if (e != hipSuccess) return hip_status(e, "seal");
  if (nbad) return Status::Corruption("log record outside the image");  // cannot happen
  for (size_t i = 0; i < count; i++) {  // EncodeFixed32 (util/coding.cc)
    char* h = &dest_[headers_[sealed_ + i]];
    for (int k = 0; k < 4; k++) h[k] = (char)(masked[i] >> (8 * k));
  }
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
  {  // pass 1: every header the reader could check (all checksums assumed good)
    Walk collect(img, size_, initial_offset_, nullptr, &headers_, nullptr, nullptr);
    std::string rec;
    uint64_t off = 0;
    while (collect.ReadRecord(&rec, &off)) {
    }
  }
  ok_.assign(headers_.size(), 0);
  if (!headers_.empty()) {  // one GPU batch for all of them
    DeviceLog d;
    Status s = stage(device, file_, size_, headers_.data(), headers_.size(), headers_.size(), &d);
    if (!s.ok()) return s;
    if (lsbm_log_verify_dev(d.image, size_, d.headers, headers_.size(),
                            static_cast<uint8_t*>(d.aux), d.nbad, d.stream.get()) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    hipError_t e = d.bounce.to_host(ok_.data(), d.aux, headers_.size(), d.stream.get());
    if (e != hipSuccess) return hip_status(e, "verify");
  }
  // pass 2 (ReadRecord): the reader itself, with the GPU's verdicts
  walk_ = new Walk(img, size_, initial_offset_, reporter_, nullptr, &headers_, &ok_);
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
