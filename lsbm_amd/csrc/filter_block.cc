// filter_block.cc -- include/lsbm/filter_block.h on top of the C ABI.
//
// Builder: the reference's layout decisions (which keys form which filter,
// table/filter_block.cc:22-28, 52-76) are made on the host as keys arrive;
// they depend only on block offsets and key counts, so the whole block layout
// is known before any hashing.  Finish stages every builder's keys once, runs
// one lsbm_bloom_build_dev over all their filters, and appends the offset
// array, array_offset and base_lg (:41-49) on the host.
#include "../../include/lsbm/filter_block.h"

#include <hip/hip_runtime_api.h>
#include <string.h>

#include <memory>

#include "../../include/lsbm_bloom.h"
#include "host_session.h"

namespace lsbm {

namespace {

constexpr uint64_t kFilterBase = 1ull << LSBM_FILTER_BASE_LG;  // table/filter_block.cc:14-16

void put_fixed32(std::string* dst, uint32_t v) {  // util/coding.cc PutFixed32
  const char b[4] = {(char)(v & 0xff), (char)((v >> 8) & 0xff), (char)((v >> 16) & 0xff),
                     (char)(v >> 24)};
  dst->append(b, 4);
}

}  // namespace

FilterBlockBuilder::FilterBlockBuilder(const BloomOptions& options)
    : options_(options), pending_(0) {}

void FilterBlockBuilder::StartBlock(uint64_t block_offset) {
  const uint64_t filter_index = block_offset / kFilterBase;
  while (filter_index > filters_.size()) GenerateFilter();
}

void FilterBlockBuilder::AddKey(const char* key, size_t n) {
  starts_.push_back(keys_.size());
  keys_.append(key, n);
}

void FilterBlockBuilder::GenerateFilter() {
  filters_.push_back(Range{pending_, (uint64_t)starts_.size()});
  pending_ = starts_.size();
}

Status FilterBlockBuilder::Finish(int device, std::string* result) {
  FilterBlockBuilder* self = this;
  return FinishFilterBlocks(device, &self, 1, result);
}

Status FinishFilterBlocks(int device, FilterBlockBuilder* const* builders, size_t n,
                          std::string* results) {
  if (n == 0) return Status::OK();
  HostTiming tm("FinishFilterBlocks");  // (LSBM_HOST_TIMING=1: prep = layout, copy = uploads,
                                        //  enqueue = build, wait = download, post = blocks)
  double ph = HostTiming::now();
  auto lap = [&](HostTiming::Phase p) {
    const double t = HostTiming::now();
    tm.add(p, t - ph);
    ph = t;
  };
  const int bpk = builders[0]->options_.bits_per_key;
  const bool internal = builders[0]->options_.internal_keys;
  if (bpk < 0) return Status::InvalidArgument("bits_per_key < 0");
  // host layout of every block.  The builders' keys are not concatenated on
  // the host: they are gathered straight into the staging chunks on their way
  // to the device, and only the key offsets are rebased here (into a vector
  // sized once, builder by builder on the pool).  (Concatenating 240 MB of
  // keys for a 10M-key compaction cost more than the rest of the call.)
  uint64_t total_keys = 0, total_bytes = 0;
  for (size_t t = 0; t < n; t++) {
    FilterBlockBuilder& b = *builders[t];
    if (b.options_.bits_per_key != bpk || b.options_.internal_keys != internal)
      return Status::InvalidArgument("one bits_per_key and key kind per batch");
    if (b.pending_ < b.starts_.size()) b.GenerateFilter();  // Finish, :37-39
    total_keys += b.starts_.size();
    total_bytes += b.keys_.size();
  }
  // (no zero fill: every entry is written, in parallel, by the pass below)
  std::unique_ptr<uint64_t[]> key_offs(new uint64_t[total_keys + 1]);
  std::vector<uint64_t> first, out_off, byte_base(n), key_base(n);
  std::vector<uint64_t> data_base(n), data_size(n);
  std::vector<std::vector<uint32_t>> offsets(n);
  uint64_t out_total = 0, bytes_so_far = 0, keys_so_far = 0;
  for (size_t t = 0; t < n; t++) {
    byte_base[t] = bytes_so_far;
    key_base[t] = keys_so_far;
    bytes_so_far += builders[t]->keys_.size();
    keys_so_far += builders[t]->starts_.size();
  }
  // the rebased key offsets, builder by builder on the worker pool
  parallel_for(n, [&](size_t t) {
    const std::vector<uint64_t>& st = builders[t]->starts_;
    uint64_t* o = key_offs.get() + key_base[t];
    for (size_t k = 0; k < st.size(); k++) o[k] = byte_base[t] + st[k];
  });
  for (size_t t = 0; t < n; t++) {
    FilterBlockBuilder& b = *builders[t];
    const uint64_t kb = key_base[t];
    uint64_t size = 0;
    for (const auto& r : b.filters_) {
      offsets[t].push_back((uint32_t)size);  // filter_offsets_ (:56, :70)
      if (r.hi > r.lo) {
        first.push_back(kb + r.lo);
        out_off.push_back(out_total + size);
        size += lsbm_bloom_filter_bytes(r.hi - r.lo, bpk);
      }
    }
    data_base[t] = out_total;
    data_size[t] = size;
    out_total += size;
  }
  key_offs[total_keys] = total_bytes;
  first.push_back(total_keys);  // filters cover every key, in order
  std::unique_ptr<char[]> data(new char[out_total ? out_total : 1]);
  const size_t nf = out_off.size();
  lap(HostTiming::kPrep);
  if (nf) {  // one launch on the device's session (host_session.h)
    SessionLease ss;
    Status s = ss.Open(device);
    if (!s.ok()) return s;
    void *d_keys, *d_offs, *d_first, *d_out_off, *d_out;
    hipError_t e = ss->scratch(0, total_bytes ? total_bytes : 1, &d_keys);
    if (e == hipSuccess) e = ss->scratch(1, (total_keys + 1) * sizeof(uint64_t), &d_offs);
    if (e == hipSuccess) e = ss->scratch(2, first.size() * sizeof(uint64_t), &d_first);
    if (e == hipSuccess) e = ss->scratch(3, out_off.size() * sizeof(uint64_t), &d_out_off);
    if (e == hipSuccess) e = ss->scratch(4, out_total, &d_out);
    std::vector<HostSession::Piece> pieces(n);  // every builder's keys, back to back: one gather
    for (size_t t = 0; t < n; t++) pieces[t] = HostSession::Piece{builders[t]->keys_.data(), builders[t]->keys_.size()};
    if (e == hipSuccess) e = ss->upload_pieces(d_keys, pieces.data(), n);
    if (e == hipSuccess) e = ss->upload(d_offs, key_offs.get(), (total_keys + 1) * sizeof(uint64_t));
    if (e == hipSuccess) e = ss->upload(d_first, first.data(), first.size() * sizeof(uint64_t));
    if (e == hipSuccess) e = ss->upload(d_out_off, out_off.data(), out_off.size() * sizeof(uint64_t));
    if (e != hipSuccess) return hip_status(e, "staging");
    lap(HostTiming::kCopy);
    if (lsbm_bloom_build_dev(static_cast<const uint8_t*>(d_keys), static_cast<const uint64_t*>(d_offs),
                             internal ? LSBM_INTERNAL_KEY_SUFFIX : 0,
                             static_cast<const uint64_t*>(d_first), static_cast<const uint64_t*>(d_out_off),
                             nf, bpk, static_cast<uint8_t*>(d_out), ss->stream()) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    lap(HostTiming::kEnqueue);
    e = ss->download(data.get(), d_out, out_total);
    if (e != hipSuccess) return hip_status(e, "filters");
    lap(HostTiming::kWait);
  }
  for (size_t t = 0; t < n; t++) {  // :41-49
    std::string& r = results[t];
    r.reserve(data_size[t] + 4 * offsets[t].size() + 5);
    r.assign(data.get() + data_base[t], data_size[t]);
    for (uint32_t o : offsets[t]) put_fixed32(&r, o);
    put_fixed32(&r, (uint32_t)data_size[t]);
    r.push_back((char)LSBM_FILTER_BASE_LG);
  }
  lap(HostTiming::kPost);
  return Status::OK();
}

FilterBlockReader::FilterBlockReader(const BloomOptions& options, const char* contents, size_t n)
    : options_(options), contents_(contents), size_(n) {}

Status FilterBlockReader::KeyMayMatch(int device, const uint64_t* block_offsets, const char* keys,
                                      const uint64_t* key_offsets, size_t n,
                                      std::vector<uint8_t>* may) const {
  may->assign(n, 1);
  if (n == 0) return Status::OK();
  if (!block_offsets || !keys || !key_offsets) return Status::InvalidArgument("null pointer");
  SessionLease ss;
  Status s = ss.Open(device);
  if (!s.ok()) return s;
  std::vector<uint64_t> handles(2 * n), offs(n + 1);
  for (size_t i = 0; i < n; i++) {
    handles[2 * i] = 0;
    handles[2 * i + 1] = size_;
  }
  for (size_t i = 0; i <= n; i++) offs[i] = key_offsets[i] - key_offsets[0];
  void *d_block, *d_keys, *d_may, *d_handles, *d_data, *d_offs;
  hipError_t e = ss->scratch(0, size_, &d_block);
  if (e == hipSuccess) e = ss->scratch(1, handles.size() * sizeof(uint64_t), &d_handles);
  if (e == hipSuccess) e = ss->scratch(2, n * sizeof(uint64_t), &d_data);
  if (e == hipSuccess) e = ss->scratch(3, offs[n], &d_keys);
  if (e == hipSuccess) e = ss->scratch(4, offs.size() * sizeof(uint64_t), &d_offs);
  if (e == hipSuccess) e = ss->scratch(5, n, &d_may);
  if (e == hipSuccess) e = ss->upload(d_block, contents_, size_);
  if (e == hipSuccess) e = ss->upload(d_handles, handles.data(), handles.size() * sizeof(uint64_t));
  if (e == hipSuccess) e = ss->upload(d_data, block_offsets, n * sizeof(uint64_t));
  if (e == hipSuccess) e = ss->upload(d_keys, keys + key_offsets[0], offs[n]);
  if (e == hipSuccess) e = ss->upload(d_offs, offs.data(), offs.size() * sizeof(uint64_t));
  if (e != hipSuccess) return hip_status(e, "staging");
  if (lsbm_filter_block_may_match_dev(static_cast<const uint8_t*>(d_block),
                                      static_cast<const uint64_t*>(d_handles),
                                      static_cast<const uint64_t*>(d_data),
                                      static_cast<const uint8_t*>(d_keys),
                                      static_cast<const uint64_t*>(d_offs),
                                      options_.internal_keys ? LSBM_INTERNAL_KEY_SUFFIX : 0, n,
                                      options_.bits_per_key, options_.bloom_bits_use,
                                      static_cast<uint8_t*>(d_may), nullptr, ss->stream()) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  e = ss->download(may->data(), d_may, n);
  return e == hipSuccess ? Status::OK() : hip_status(e, "lookups");
}

}  // namespace lsbm
