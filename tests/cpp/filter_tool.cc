// filter_tool -- drives include/lsbm/filter_block.h for tests/test_bloom.py.
//
//   filter_tool build <keys.bin> <offs.bin> <blocks.bin> <out.bin> <bits_per_key> <strip> [copies]
//       keys[offs[i], offs[i+1]) (offs: LE uint64), blocks.bin = LE uint64
//       [n, start_0..start_{n-1}, first_0..first_n]: StartBlock(start_b) then
//       AddKey for keys [first_b, first_b+1); Finish on GPU 0.  With copies > 1
//       the same sequence is fed to `copies` builders finished together by
//       FinishFilterBlocks; every result must be identical.  Writes the block.
//   filter_tool probe <block.bin> <keys.bin> <offs.bin> <data_offsets.bin> <bits_per_key>
//                     <bloom_bits_use> <strip>
//       FilterBlockReader::KeyMayMatch for every key on GPU 0; prints 0/1 per key.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "lsbm/filter_block.h"

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

static std::vector<uint64_t> u64s(const std::string& s) {
  std::vector<uint64_t> v(s.size() / 8);
  if (!v.empty()) memcpy(v.data(), s.data(), v.size() * 8);
  return v;
}

int main(int argc, char** argv) {
  if (argc >= 8 && !strcmp(argv[1], "build")) {
    const std::string keys = slurp(argv[2]);
    const std::vector<uint64_t> offs = u64s(slurp(argv[3])), blk = u64s(slurp(argv[4]));
    lsbm::BloomOptions opt;
    opt.bits_per_key = atoi(argv[6]);
    opt.internal_keys = atoi(argv[7]) == 8;
    const size_t copies = argc > 8 ? strtoul(argv[8], nullptr, 10) : 1;
    const size_t n = blk[0];
    std::vector<std::unique_ptr<lsbm::FilterBlockBuilder>> b;
    std::vector<lsbm::FilterBlockBuilder*> raw;
    for (size_t c = 0; c < copies; c++) {
      b.emplace_back(new lsbm::FilterBlockBuilder(opt));
      raw.push_back(b.back().get());
    }
    for (auto& x : b)
      for (size_t i = 0; i < n; i++) {
        x->StartBlock(blk[1 + i]);
        for (uint64_t k = blk[1 + n + i]; k < blk[2 + n + i]; k++)
          x->AddKey(keys.data() + offs[k], offs[k + 1] - offs[k]);
      }
    std::vector<std::string> out(copies);
    lsbm::Status s = copies == 1 ? raw[0]->Finish(0, &out[0])
                                 : lsbm::FinishFilterBlocks(0, raw.data(), copies, out.data());
    if (!s.ok()) {
      fprintf(stderr, "%s\n", s.ToString().c_str());
      return 1;
    }
    for (size_t c = 1; c < copies; c++)
      if (out[c] != out[0]) {
        fprintf(stderr, "builder %zu differs\n", c);
        return 1;
      }
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(out[0].data(), 1, out[0].size(), f) != out[0].size()) return 2;
    fclose(f);
    return 0;
  }
  if (argc == 9 && !strcmp(argv[1], "probe")) {
    const std::string block = slurp(argv[2]), keys = slurp(argv[3]);
    const std::vector<uint64_t> offs = u64s(slurp(argv[4])), data = u64s(slurp(argv[5]));
    lsbm::BloomOptions opt;
    opt.bits_per_key = atoi(argv[6]);
    opt.bloom_bits_use = atoi(argv[7]);
    opt.internal_keys = atoi(argv[8]) == 8;
    lsbm::FilterBlockReader r(opt, block.data(), block.size());
    std::vector<uint8_t> may;
    lsbm::Status s = r.KeyMayMatch(0, data.data(), keys.data(), offs.data(), data.size(), &may);
    if (!s.ok()) {
      fprintf(stderr, "%s\n", s.ToString().c_str());
      return 1;
    }
    std::string line;
    for (uint8_t m : may) line.push_back(m ? '1' : '0');
    printf("%s\n", line.c_str());
    return 0;
  }
  fprintf(stderr, "usage: filter_tool build|probe ...\n");
  return 2;
}
