// ref_log_shim.cc -- TEST INFRASTRUCTURE ONLY.  A C-ABI shim compiled together
// with the *reference's own* common/log_writer.cc, common/log_reader.cc and
// util/{crc32c,coding,status,env}.cc (never copied into this repo) into
// oracle/_ref/libref_log.so (oracle/Makefile, target `reflog`), so that the
// WAL fixtures of tests/golden/make_log_fixture.py are written and read by
// the reference's log::Writer and log::Reader themselves.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "leveldb/env.h"
#include "log_reader.h"  // common/, resolved against -I/root/reference/common
#include "log_writer.h"
#include "util/crc32c.h"

namespace {

// In-memory WritableFile / SequentialFile for the reference's Writer / Reader.
class StringSink : public leveldb::WritableFile {
 public:
  std::string data;
  leveldb::Status Append(const leveldb::Slice& s) override {
    data.append(s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }
};

class StringSource : public leveldb::SequentialFile {
 public:
  StringSource(const char* p, size_t n) : p_(p), n_(n), pos_(0) {}
  leveldb::Status Read(size_t n, leveldb::Slice* result, char* scratch) override {
    const size_t k = n < n_ - pos_ ? n : n_ - pos_;
    memcpy(scratch, p_ + pos_, k);
    *result = leveldb::Slice(scratch, k);
    pos_ += k;
    return leveldb::Status::OK();
  }
  leveldb::Status Skip(uint64_t n) override {
    pos_ = n > n_ - pos_ ? n_ : pos_ + n;
    return leveldb::Status::OK();
  }

 private:
  const char* p_;
  size_t n_, pos_;
};

// Events in the text form tests/cpp/log_tool.cc prints:
//   R <length> <crc32c of the record, hex> <LastRecordOffset>
//   D <bytes> <Status::ToString()>
class Events : public leveldb::log::Reader::Reporter {
 public:
  std::string text;
  void Corruption(size_t bytes, const leveldb::Status& s) override {
    char buf[64];
    snprintf(buf, sizeof(buf), "D %zu ", bytes);
    text += buf + s.ToString() + "\n";
  }
};

size_t out_copy(const std::string& s, char* out, size_t cap) {
  if (s.size() <= cap) memcpy(out, s.data(), s.size());
  return s.size();
}

}  // namespace

extern "C" {

// log::Writer::AddRecord for records payload[offs[i], offs[i+1]); the bytes
// the writer appended go to out (returns their count; copies only if <= cap).
size_t ref_log_write(const char* payload, const uint64_t* offs, size_t n, char* out, size_t cap) {
  StringSink sink;
  leveldb::log::Writer w(&sink);
  for (size_t i = 0; i < n; i++)
    w.AddRecord(leveldb::Slice(payload + offs[i], offs[i + 1] - offs[i]));
  return out_copy(sink.data, out, cap);
}

// log::Reader(file, reporter, checksum=true, initial_offset) over image[0, n):
// every ReadRecord result and Reporter call, in order, as event text.
size_t ref_log_read_from(const char* image, size_t n, uint64_t initial_offset, char* out,
                         size_t cap) {
  StringSource src(image, n);
  Events ev;
  leveldb::log::Reader r(&src, &ev, true, initial_offset);
  leveldb::Slice rec;
  std::string scratch;
  while (r.ReadRecord(&rec, &scratch)) {
    char buf[96];
    snprintf(buf, sizeof(buf), "R %zu %08x %llu\n", rec.size(),
             leveldb::crc32c::Value(rec.data(), rec.size()),
             (unsigned long long)r.LastRecordOffset());
    ev.text += buf;
  }
  return out_copy(ev.text, out, cap);
}

size_t ref_log_read(const char* image, size_t n, char* out, size_t cap) {
  return ref_log_read_from(image, n, 0, out, cap);
}

uint32_t ref_log_value(const char* p, size_t n) { return leveldb::crc32c::Value(p, n); }

}  // extern "C"
