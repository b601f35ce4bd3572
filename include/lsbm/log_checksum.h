// include/lsbm/log_checksum.h -- C++ host API for lsbm's WAL / MANIFEST logs
// (common/log_format.h, common/log_writer.cc, common/log_reader.cc) with the
// record CRCs computed in one GPU batch per call.
//
//   BatchWriter   frames records exactly like log::Writer::AddRecord
//                 (common/log_writer.cc:27-73: same FULL/FIRST/MIDDLE/LAST
//                 fragments, same zero-filled block trailers), but defers the
//                 header CRCs (:86-88); Seal() computes all pending ones on
//                 the GPU (lsbm_log_seal_dev).  This is a group commit: many
//                 AddRecord calls, one CRC batch.
//   ReadLog       what DBImpl::RecoverLogFile / VersionSet::Recover get from
//                 log::Reader(file, reporter, checksum=true, initial_offset)
//                 (lsbm/db_impl.cc:428, lsbm/version_set.cc:2026): the same
//                 records in the same order and the same Reporter::Corruption
//                 calls (bytes, status), with every physical record's
//                 checksum (common/log_reader.cc:228-242) verified in one GPU
//                 batch (lsbm_log_verify_dev).
//
// No HIP types in this header; the image lives in host memory and is staged
// to `device` for the CRC work only.
#ifndef LSBM_LOG_CHECKSUM_H_
#define LSBM_LOG_CHECKSUM_H_

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "lsbm/status.h"

namespace lsbm {
namespace log {

// common/log_format.h:14-30
enum RecordType {
  kZeroType = 0,  // reserved for preallocated files
  kFullType = 1,
  kFirstType = 2,
  kMiddleType = 3,
  kLastType = 4
};
static const int kMaxRecordType = kLastType;
static const int kBlockSize = 32768;
static const int kHeaderSize = 4 + 2 + 1;  // crc, length, type

class BatchWriter {
 public:
  // A writer over an empty destination, like log::Writer(dest)
  // (common/log_writer.cc:15-17: block_offset_ starts at 0).
  BatchWriter();

  // Frames `n` bytes as one logical record (common/log_writer.cc:27-73).  The
  // CRC fields of its headers stay zero until Seal().
  void AddRecord(const char* data, size_t n);

  // Computes the CRC of every header added since the last Seal() on the GPU
  // and stores Mask(crc) in it (common/log_writer.cc:86-88).
  Status Seal(int device);

  // The bytes log::Writer would have appended to its WritableFile so far.
  const std::string& contents() const { return dest_; }
  // Offsets of every physical record header in contents().
  const std::vector<uint64_t>& headers() const { return headers_; }

 private:
  std::string dest_;
  int block_offset_;
  std::vector<uint64_t> headers_;
  size_t sealed_;  // headers_[0, sealed_) carry their CRC
};

// log::Reader::Reporter (common/log_reader.h:23-30).
class Reporter {
 public:
  virtual ~Reporter() {}
  // Some corruption was detected; `bytes` is the approximate number dropped.
  virtual void Corruption(size_t bytes, const Status& status) = 0;
};

// log::Reader (common/log_reader.h:20-103) over an in-memory log file image
// file[0, n), with checksum = true.  lsbm's recovery reads from offset 0
// (lsbm/db_impl.cc:428, lsbm/version_set.cc:2026); a non-zero initial_offset
// behaves as the reference's: reading starts at the block holding it
// (SkipToInitialBlock, common/log_reader.cc:35-57), physical records that
// begin before it are skipped, and drops before it are not reported
// (:171-176, :247-251).  Verify() checks every physical record's CRC in one
// GPU batch; ReadRecord() then returns the same records, with the same
// LastRecordOffset() and the same reporter->Corruption calls, in the same
// order as the reference reader.  `file` and `reporter` must outlive it.
class Walk;
class BatchReader {
 public:
  BatchReader(const char* file, size_t n, Reporter* reporter, uint64_t initial_offset = 0);
  ~BatchReader();

  // The GPU batch (lsbm_log_verify_dev).  Must precede ReadRecord; a non-OK
  // status means the device work failed, never that a record is corrupt.
  Status Verify(int device);

  // common/log_reader.cc:59-162: false at the end of the input.  *record stays
  // valid until the next call.
  bool ReadRecord(std::string* record);
  uint64_t LastRecordOffset() const { return last_record_offset_; }

 private:
  BatchReader(const BatchReader&);
  void operator=(const BatchReader&);
  const char* file_;
  size_t size_;
  Reporter* reporter_;
  uint64_t initial_offset_;
  std::vector<uint64_t> headers_;  // every header the reader may check
  std::vector<uint8_t> ok_;        // their CRC verdicts
  Walk* walk_;
  uint64_t last_record_offset_;
};

// Convenience: every record of the image (and its offset), as a recovery
// loop over BatchReader::ReadRecord collects them.
Status ReadLog(int device, const char* file, size_t n, Reporter* reporter,
               std::vector<std::string>* records, std::vector<uint64_t>* offsets,
               uint64_t initial_offset = 0);

}  // namespace log
}  // namespace lsbm

#endif  // LSBM_LOG_CHECKSUM_H_
