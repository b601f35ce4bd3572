// status.cc -- lsbm::Status::ToString (include/lsbm/status.h), the text of
// leveldb::Status::ToString (util/status.cc) for the codes this library uses.
#include "../../include/lsbm/status.h"

namespace lsbm {

std::string Status::ToString() const {
  switch (code_) {
    case kOk: return "OK";
    case kCorruption: return "Corruption: " + msg_;
    case kInvalidArgument: return "Invalid argument: " + msg_;
    default: return "IO error: " + msg_;
  }
}

}  // namespace lsbm
