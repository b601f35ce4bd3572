// ref_bloom_shim.cc -- TEST INFRASTRUCTURE ONLY.  A C-ABI shim compiled with
// the *reference's own* util/hash.cc, util/bloom.cc, util/filter_policy.cc,
// table/filter_block.cc, util/coding.cc and common/params.cc (never copied
// into this repo) into oracle/_ref/libref_bloom.so (oracle/Makefile, target
// `refbloom`), so that tests/golden/make_bloom_fixture.py records what the
// reference's Hash, BloomFilterPolicy, FilterBlockBuilder and
// FilterBlockReader themselves produce.
//
// `strip` emulates InternalFilterPolicy (common/dbformat.cc:105-119: every key
// loses its 8-byte sequence/type suffix before the user policy sees it); the
// real db_bench SSTable fixture pins that wrapper with the reference's own code.
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "leveldb/filter_policy.h"
#include "leveldb/params.h"
#include "leveldb/slice.h"
#include "table/filter_block.h"
#include "util/hash.h"

namespace {

class StripPolicy : public leveldb::FilterPolicy {  // InternalFilterPolicy's key handling
 public:
  StripPolicy(const leveldb::FilterPolicy* user, size_t strip) : user_(user), strip_(strip) {}
  const char* Name() const override { return user_->Name(); }
  void CreateFilter(const leveldb::Slice* keys, int n, std::string* dst) const override {
    std::vector<leveldb::Slice> k(keys, keys + n);
    for (auto& s : k) s = leveldb::Slice(s.data(), s.size() - strip_);
    user_->CreateFilter(n ? &k[0] : nullptr, n, dst);
  }
  bool KeyMayMatch(const leveldb::Slice& key, const leveldb::Slice& f) const override {
    return user_->KeyMayMatch(leveldb::Slice(key.data(), key.size() - strip_), f);
  }

 private:
  const leveldb::FilterPolicy* user_;
  size_t strip_;
};

size_t out_copy(const std::string& s, char* out, size_t cap) {
  if (s.size() <= cap) memcpy(out, s.data(), s.size());
  return s.size();
}

}  // namespace

extern "C" {

uint32_t ref_hash(const char* p, size_t n, uint32_t seed) { return leveldb::Hash(p, n, seed); }

// The read-side probe count is fixed when a policy is constructed
// (util/bloom.cc:28), from this global (common/params.cc:29).
void ref_set_bloom_bits_use(int v) { leveldb::config::bloom_bits_use = v; }

size_t ref_create_filter(int bits_per_key, const char* keys, const uint64_t* offs, int n,
                         char* out, size_t cap) {
  const leveldb::FilterPolicy* p = leveldb::NewBloomFilterPolicy(bits_per_key);
  std::vector<leveldb::Slice> k(n);
  for (int i = 0; i < n; i++) k[i] = leveldb::Slice(keys + offs[i], offs[i + 1] - offs[i]);
  std::string dst;
  p->CreateFilter(n ? &k[0] : nullptr, n, &dst);
  delete p;
  return out_copy(dst, out, cap);
}

int ref_key_may_match(int bits_per_key, const char* key, size_t kn, const char* filter,
                      size_t len) {
  const leveldb::FilterPolicy* p = leveldb::NewBloomFilterPolicy(bits_per_key);
  const bool r = p->KeyMayMatch(leveldb::Slice(key, kn), leveldb::Slice(filter, len));
  delete p;
  return r ? 1 : 0;
}

size_t ref_filter_block_build(int bits_per_key, int strip, const char* keys,
                              const uint64_t* key_offs, const uint64_t* block_start,
                              const uint64_t* block_first, size_t n_blocks, char* out,
                              size_t cap) {
  const leveldb::FilterPolicy* user = leveldb::NewBloomFilterPolicy(bits_per_key);
  StripPolicy policy(user, (size_t)strip);
  std::string r;
  {
    leveldb::FilterBlockBuilder b(&policy);
    for (size_t i = 0; i < n_blocks; i++) {
      b.StartBlock(block_start[i]);
      for (uint64_t k = block_first[i]; k < block_first[i + 1]; k++)
        b.AddKey(leveldb::Slice(keys + key_offs[k], key_offs[k + 1] - key_offs[k]));
    }
    const leveldb::Slice s = b.Finish();
    r.assign(s.data(), s.size());
  }
  delete user;
  return out_copy(r, out, cap);
}

int ref_filter_block_may_match(int bits_per_key, int strip, const char* contents, size_t n,
                               uint64_t block_offset, const char* key, size_t kn) {
  const leveldb::FilterPolicy* user = leveldb::NewBloomFilterPolicy(bits_per_key);
  StripPolicy policy(user, (size_t)strip);
  bool r;
  {
    leveldb::FilterBlockReader reader(&policy, leveldb::Slice(contents, n));
    r = reader.KeyMayMatch(block_offset, leveldb::Slice(key, kn));
  }
  delete user;
  return r ? 1 : 0;
}

// Batch drivers for the CPU baseline (tools/bench_bloom.py): the reference's
// CreateFilter over n_filters filters of keys [first[f], first[f+1]) (one
// policy object, as a TableBuilder holds), and KeyMayMatch of key i against
// filter fidx[i] (filters at fo[f], fo[f+1]); returns the number of matches.
size_t ref_create_filters(int bits_per_key, const char* keys, const uint64_t* offs,
                          const uint64_t* first, size_t n_filters, char* out, uint64_t* fo) {
  const leveldb::FilterPolicy* p = leveldb::NewBloomFilterPolicy(bits_per_key);
  std::string dst;
  std::vector<leveldb::Slice> k;
  fo[0] = 0;
  for (size_t f = 0; f < n_filters; f++) {
    k.clear();
    for (uint64_t i = first[f]; i < first[f + 1]; i++)
      k.push_back(leveldb::Slice(keys + offs[i], offs[i + 1] - offs[i]));
    p->CreateFilter(k.empty() ? nullptr : &k[0], (int)k.size(), &dst);
    fo[f + 1] = dst.size();
  }
  delete p;
  memcpy(out, dst.data(), dst.size());
  return dst.size();
}

size_t ref_may_match_batch(int bits_per_key, const char* keys, const uint64_t* offs, size_t n,
                           const char* filters, const uint64_t* fo, const uint64_t* fidx) {
  const leveldb::FilterPolicy* p = leveldb::NewBloomFilterPolicy(bits_per_key);
  size_t hits = 0;
  for (size_t i = 0; i < n; i++) {
    const uint64_t f = fidx[i];
    hits += p->KeyMayMatch(leveldb::Slice(keys + offs[i], offs[i + 1] - offs[i]),
                           leveldb::Slice(filters + fo[f], fo[f + 1] - fo[f]));
  }
  delete p;
  return hits;
}

}  // extern "C"
