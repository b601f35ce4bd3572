// Compiles against include/util/crc32c.h exactly as lsbm's table/ and
// common/log_* do (#include "util/crc32c.h", namespace leveldb::crc32c) and
// links liblsbm_crc32c.so: proves the drop-in keeps the reference's API and
// its exported symbol _ZN7leveldb6crc32c6ExtendEjPKcm.
// Mirrors the call pattern of TableBuilder::WriteRawBlock
// (table/table_builder.cc:245-249) and log::Writer (common/log_writer.cc:18-21,86-87).
#include <stdio.h>
#include <string.h>

#include <string>

#include "util/crc32c.h"

using namespace leveldb;

static int fails = 0;
#define EXPECT(c)                                              \
  do {                                                         \
    if (!(c)) {                                                \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
      fails++;                                                 \
    }                                                          \
  } while (0)

int main() {
  char buf[32];
  memset(buf, 0, sizeof(buf));
  EXPECT(crc32c::Value(buf, 32) == 0x8a9136aau);
  memset(buf, 0xff, sizeof(buf));
  EXPECT(crc32c::Value(buf, 32) == 0x62a8ab43u);
  for (int i = 0; i < 32; i++) buf[i] = (char)i;
  EXPECT(crc32c::Value(buf, 32) == 0x46dd794eu);
  EXPECT(crc32c::Value("123456789", 9) == 0xe3069283u);
  EXPECT(crc32c::Value("", 0) == 0);
  EXPECT(crc32c::Extend(crc32c::Value("hello ", 6), "world", 5) == crc32c::Value("hello world", 11));
  const uint32_t foo = crc32c::Value("foo", 3);
  EXPECT(crc32c::Mask(foo) != foo);
  EXPECT(crc32c::Mask(foo) == 0xfebe8a61u);
  EXPECT(crc32c::Mask(crc32c::Mask(foo)) == 0xb746e855u);
  EXPECT(crc32c::Unmask(crc32c::Mask(foo)) == foo);
  EXPECT(crc32c::Unmask(crc32c::Mask(crc32c::Mask(foo))) == crc32c::Mask(foo));
  // WriteRawBlock pattern: block then 1-byte type extension == Value(block||type)
  std::string block(4118, 'x');
  for (size_t i = 0; i < block.size(); i++) block[i] = (char)(' ' + (i * 7919) % 95);
  char trailer[1] = {1};
  uint32_t crc = crc32c::Value(block.data(), block.size());
  crc = crc32c::Extend(crc, trailer, 1);
  std::string with_type = block + std::string(trailer, 1);
  EXPECT(crc == crc32c::Value(with_type.data(), with_type.size()));
  // alignment independence (util/crc32c.cc:304-313 byte-steps to alignment)
  std::string big(70001, 0);
  for (size_t i = 0; i < big.size(); i++) big[i] = (char)(i * 2654435761u >> 13);
  const uint32_t ref = crc32c::Value(big.data() + 1, 70000);
  std::string copy(big.data() + 1, 70000);
  EXPECT(crc32c::Value(copy.data(), copy.size()) == ref);
  // log::Writer pattern: type_crc_ then Extend over the payload
  char t = 1;
  EXPECT(crc32c::Extend(crc32c::Value(&t, 1), "payload", 7) == crc32c::Value("\x01payload", 8));
  printf("%s\n", fails ? "FAILED" : "OK");
  return fails ? 1 : 0;
}
