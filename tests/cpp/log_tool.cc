// log_tool -- drives include/lsbm/log_checksum.h for tests/test_log.py.
//
//   log_tool layout <payload.bin> <offs.bin> <out.bin>
//       frame records payload[offs[i], offs[i+1]) (offs: n+1 LE uint64) with
//       BatchWriter, no CRCs (host only); prints the header offsets
//   log_tool write <payload.bin> <offs.bin> <out.bin> <batch>
//       same, sealing on GPU 0 after every `batch` records (group commits)
//   log_tool read <image.bin>
//       ReadLog on GPU 0; prints, in order,
//         R <length> <crc32c of the record, hex> <record offset>
//         D <bytes> <status>          (each Reporter::Corruption call)
//       -- the same text oracle/ref_log_shim.cc prints for the reference's
//       log::Reader.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "lsbm/log_checksum.h"
#include "util/crc32c.h"

static std::string slurp(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(2);
  }
  std::string s;
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, k);
  fclose(f);
  return s;
}

static void spit(const char* path, const std::string& s) {
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(s.data(), 1, s.size(), f) != s.size()) {
    perror(path);
    exit(2);
  }
  fclose(f);
}

class PrintReporter : public lsbm::log::Reporter {
 public:
  void Corruption(size_t bytes, const lsbm::Status& s) override {
    printf("D %zu %s\n", bytes, s.ToString().c_str());
  }
};

int main(int argc, char** argv) {
  if (argc >= 5 && (!strcmp(argv[1], "layout") || !strcmp(argv[1], "write"))) {
    const std::string payload = slurp(argv[2]), offs_raw = slurp(argv[3]);
    std::vector<uint64_t> offs(offs_raw.size() / 8);
    memcpy(offs.data(), offs_raw.data(), offs.size() * 8);
    const bool seal = !strcmp(argv[1], "write");
    const size_t batch = seal && argc > 5 ? strtoul(argv[5], nullptr, 10) : 0;
    lsbm::log::BatchWriter w;
    for (size_t i = 0; i + 1 < offs.size(); i++) {
      w.AddRecord(payload.data() + offs[i], offs[i + 1] - offs[i]);
      if (batch && (i + 1) % batch == 0) {
        lsbm::Status s = w.Seal(0);
        if (!s.ok()) {
          fprintf(stderr, "%s\n", s.ToString().c_str());
          return 1;
        }
      }
    }
    if (seal) {
      lsbm::Status s = w.Seal(0);
      if (!s.ok()) {
        fprintf(stderr, "%s\n", s.ToString().c_str());
        return 1;
      }
    }
    spit(argv[4], w.contents());
    for (uint64_t h : w.headers()) printf("%llu\n", (unsigned long long)h);
    return 0;
  }
  if ((argc == 3 || argc == 4) && !strcmp(argv[1], "read")) {
    const std::string img = slurp(argv[2]);
    const uint64_t initial_offset = argc == 4 ? strtoull(argv[3], nullptr, 10) : 0;
    PrintReporter rep;  // prints each drop as it happens, between the records
    lsbm::log::BatchReader reader(img.data(), img.size(), &rep, initial_offset);
    lsbm::Status s = reader.Verify(0);
    if (!s.ok()) {
      fprintf(stderr, "%s\n", s.ToString().c_str());
      return 1;
    }
    std::string record;
    while (reader.ReadRecord(&record))
      printf("R %zu %08x %llu\n", record.size(),
             leveldb::crc32c::Value(record.data(), record.size()),
             (unsigned long long)reader.LastRecordOffset());
    return 0;
  }
  fprintf(stderr, "usage: log_tool layout|write <payload> <offs> <out> [batch] | read <image> [initial_offset]\n");
  return 2;
}
