// include/lsbm/status.h -- the subset of leveldb::Status (include/leveldb/status.h)
// that the batched table/ and log/ layers return.  Same codes, same
// ToString() text ("OK", "Corruption: <msg>", ...), so a caller that maps a
// result to the reference's Status sees identical strings.
#ifndef LSBM_STATUS_H_
#define LSBM_STATUS_H_

#include <string>

namespace lsbm {

class Status {
 public:
  Status() : code_(kOk) {}
  static Status OK() { return Status(); }
  static Status Corruption(const std::string& msg) { return Status(kCorruption, msg); }
  static Status InvalidArgument(const std::string& msg) { return Status(kInvalidArgument, msg); }
  static Status IOError(const std::string& msg) { return Status(kIOError, msg); }
  bool ok() const { return code_ == kOk; }
  bool IsCorruption() const { return code_ == kCorruption; }
  bool IsIOError() const { return code_ == kIOError; }
  std::string ToString() const;

 private:
  // include/leveldb/status.h: kOk 0, kNotFound 1, kCorruption 2, kNotSupported 3,
  // kInvalidArgument 4, kIOError 5
  enum Code { kOk = 0, kCorruption = 2, kInvalidArgument = 4, kIOError = 5 };
  Status(Code c, const std::string& m) : code_(c), msg_(m) {}
  Code code_;
  std::string msg_;
};

}  // namespace lsbm

#endif  // LSBM_STATUS_H_
