// block_compression.cc -- include/lsbm/block_compression.h on top of the C
// ABI (include/lsbm_snappy.h).  The blocks go to the device once through the
// device's HostSession (host_session.h: persistent streams and buffers, the
// caller's current device restored after), are (de)compressed there in one
// launch, and only the bytes the host keeps come back: compressed blocks are
// compacted on the device first (lsbm_gather_dev), never their capacity slots.
// WriteBlock's keep-or-not rule and the assembly of the output run on the host.
#include "../../include/lsbm/block_compression.h"

#include <hip/hip_runtime_api.h>
#include <string.h>

#include "../../include/lsbm_crc32c.h"
#include "../../include/lsbm_snappy.h"
#include "host_session.h"

namespace lsbm {

namespace {

Status check_offsets(const uint64_t* offsets, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return Status::InvalidArgument("offsets must not decrease");
  return Status::OK();
}

// Rebase offsets[0..n] to start at 0 (the staged copy starts at offsets[0]).
std::vector<uint64_t> rebased(const uint64_t* offsets, size_t n) {
  std::vector<uint64_t> r(n + 1);
  for (size_t i = 0; i <= n; i++) r[i] = offsets[i] - offsets[0];
  return r;
}

// The most a snappy stream of c bytes can expand to: its largest tag ratio
// is a 3-byte copy emitting 64 bytes (21.3x).  A preamble claiming more
// cannot be met, so RawUncompress fails it; it gets no output window.
constexpr uint64_t kMaxExpansion = 22;

}  // namespace

Status CompressBlocks(int device, const char* raw, const uint64_t* offsets, size_t n,
                      std::string* out, std::vector<uint64_t>* out_offsets,
                      std::vector<uint8_t>* types) {
  if (!offsets || !out || !out_offsets || !types) return Status::InvalidArgument("null pointer");
  out->clear();
  out_offsets->assign(1, 0);
  types->clear();
  if (n == 0) return Status::OK();
  if (!raw) return Status::InvalidArgument("null pointer");
  Status s = check_offsets(offsets, n);
  if (!s.ok()) return s;
  const std::vector<uint64_t> off = rebased(offsets, n);
  const uint64_t total = off[n];
  std::vector<uint64_t> cap(n + 1, 0);  // output slots of MaxCompressedLength bytes
  for (size_t i = 0; i < n; i++) cap[i + 1] = cap[i] + lsbm_snappy_max_compressed_length(off[i + 1] - off[i]);

  SessionLease ss;
  s = ss.Open(device);
  if (!s.ok()) return s;
  const hipStream_t st = ss->stream();
  void *d_raw, *d_off, *d_cap, *d_comp, *d_len;
  hipError_t e = ss->scratch(0, total, &d_raw);
  if (e == hipSuccess) e = ss->scratch(1, (n + 1) * sizeof(uint64_t), &d_off);
  if (e == hipSuccess) e = ss->scratch(2, (n + 1) * sizeof(uint64_t), &d_cap);
  if (e == hipSuccess) e = ss->scratch(3, cap[n], &d_comp);
  if (e == hipSuccess) e = ss->scratch(4, n * sizeof(uint64_t), &d_len);
  if (e == hipSuccess) e = ss->upload(d_raw, raw + offsets[0], total);
  if (e == hipSuccess) e = ss->upload(d_off, off.data(), (n + 1) * sizeof(uint64_t));
  if (e == hipSuccess) e = ss->upload(d_cap, cap.data(), (n + 1) * sizeof(uint64_t));
  if (e != hipSuccess) return hip_status(e, "staging");
  if (lsbm_snappy_compress_dev(d_raw, static_cast<const uint64_t*>(d_off), n, static_cast<uint8_t*>(d_comp),
                               static_cast<const uint64_t*>(d_cap), static_cast<uint64_t*>(d_len),
                               st) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  std::vector<uint64_t> clen(n);
  e = ss->download(clen.data(), d_len, n * sizeof(uint64_t));
  if (e != hipSuccess) return hip_status(e, "compress");

  // WriteBlock's rule (table/table_builder.cc:187-188), block by block: only
  // the blocks kept compressed have their bytes gathered and brought back
  types->resize(n);
  std::vector<uint64_t> keep_len(n, 0), dense(n + 1, 0);
  for (size_t i = 0; i < n; i++) {
    const uint64_t len = off[i + 1] - off[i];
    const bool keep = clen[i] != ~0ull && clen[i] < len - len / 8;
    (*types)[i] = keep ? kSnappyCompression : kNoCompression;
    keep_len[i] = keep ? clen[i] : 0;
    dense[i + 1] = dense[i] + keep_len[i];
  }
  std::string comp(dense[n], '\0');
  if (dense[n]) {
    void *d_keep, *d_dense, *d_packed;
    e = ss->scratch(4, n * sizeof(uint64_t), &d_keep);  // (d_len is no longer needed)
    if (e == hipSuccess) e = ss->scratch(5, (n + 1) * sizeof(uint64_t), &d_dense);
    if (e == hipSuccess) e = ss->scratch(6, dense[n], &d_packed);
    if (e == hipSuccess) e = ss->upload(d_keep, keep_len.data(), n * sizeof(uint64_t));
    if (e == hipSuccess) e = ss->upload(d_dense, dense.data(), (n + 1) * sizeof(uint64_t));
    if (e != hipSuccess) return hip_status(e, "staging");
    if (lsbm_gather_dev(d_comp, static_cast<const uint64_t*>(d_cap), static_cast<const uint64_t*>(d_keep), n,
                        d_packed, static_cast<const uint64_t*>(d_dense), st) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    e = ss->download(&comp[0], d_packed, dense[n]);
    if (e != hipSuccess) return hip_status(e, "compress");
  }
  out_offsets->resize(n + 1);
  out->reserve(total);
  for (size_t i = 0; i < n; i++) {
    if ((*types)[i] == kSnappyCompression)
      out->append(comp, dense[i], keep_len[i]);
    else
      out->append(raw + offsets[i], off[i + 1] - off[i]);
    (*out_offsets)[i + 1] = out->size();
  }
  return Status::OK();
}

Status UncompressBlocks(int device, const char* data, const uint64_t* offsets, const uint8_t* types,
                        size_t n, std::string* out, std::vector<uint64_t>* out_offsets,
                        std::vector<uint8_t>* ok) {
  if (!offsets || !types || !out || !out_offsets) return Status::InvalidArgument("null pointer");
  out->clear();
  out_offsets->assign(1, 0);
  if (ok) ok->assign(n, 1);
  if (n == 0) return Status::OK();
  if (!data) return Status::InvalidArgument("null pointer");
  Status s = check_offsets(offsets, n);
  if (!s.ok()) return s;

  // the snappy blocks, packed back to back for one launch
  std::vector<size_t> idx;
  std::vector<uint64_t> coff(1, 0);
  for (size_t i = 0; i < n; i++)
    if (types[i] == kSnappyCompression) {
      idx.push_back(i);
      coff.push_back(coff.back() + (offsets[i + 1] - offsets[i]));
    }
  const size_t m = idx.size();
  std::vector<uint64_t> ulen(m, 0);
  std::vector<uint8_t> len_ok(m, 0), dec_ok(m, 0);
  std::vector<uint64_t> uoff(m + 1, 0);
  std::string dec;
  if (m) {
    std::string packed;
    packed.reserve(coff[m]);
    for (size_t j = 0; j < m; j++) packed.append(data + offsets[idx[j]], offsets[idx[j] + 1] - offsets[idx[j]]);
    SessionLease ss;
    s = ss.Open(device);
    if (!s.ok()) return s;
    const hipStream_t st = ss->stream();
    void *d_comp, *d_coff, *d_ulen, *d_ok;
    hipError_t e = ss->scratch(0, coff[m], &d_comp);
    if (e == hipSuccess) e = ss->scratch(1, (m + 1) * sizeof(uint64_t), &d_coff);
    if (e == hipSuccess) e = ss->scratch(2, m * sizeof(uint64_t), &d_ulen);
    if (e == hipSuccess) e = ss->scratch(3, m, &d_ok);
    if (e == hipSuccess) e = ss->upload(d_comp, packed.data(), coff[m]);
    if (e == hipSuccess) e = ss->upload(d_coff, coff.data(), (m + 1) * sizeof(uint64_t));
    if (e != hipSuccess) return hip_status(e, "staging");
    // GetUncompressedLength sizes the output windows
    if (lsbm_snappy_uncompressed_length_dev(d_comp, static_cast<const uint64_t*>(d_coff), m,
                                            static_cast<uint64_t*>(d_ulen), static_cast<uint8_t*>(d_ok),
                                            st) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    e = ss->download(ulen.data(), d_ulen, m * sizeof(uint64_t));
    if (e == hipSuccess) e = ss->download(len_ok.data(), d_ok, m);
    if (e != hipSuccess) return hip_status(e, "uncompressed length");
    for (size_t j = 0; j < m; j++) {
      // a preamble no stream of this length can meet fails now, with no window
      if (len_ok[j] && ulen[j] > kMaxExpansion * (coff[j + 1] - coff[j])) len_ok[j] = 0;
      uoff[j + 1] = uoff[j] + (len_ok[j] ? ulen[j] : 0);
    }
    void *d_out, *d_uoff;
    e = ss->scratch(4, uoff[m], &d_out);
    if (e == hipSuccess) e = ss->scratch(5, (m + 1) * sizeof(uint64_t), &d_uoff);
    if (e == hipSuccess) e = ss->upload(d_uoff, uoff.data(), (m + 1) * sizeof(uint64_t));
    if (e != hipSuccess) return hip_status(e, "staging");
    if (lsbm_snappy_uncompress_dev(d_comp, static_cast<const uint64_t*>(d_coff), m,
                                   static_cast<uint8_t*>(d_out), static_cast<const uint64_t*>(d_uoff),
                                   static_cast<uint8_t*>(d_ok), nullptr, st) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    dec.assign(uoff[m], '\0');
    e = ss->download(dec_ok.data(), d_ok, m);
    if (e == hipSuccess && uoff[m]) e = ss->download(&dec[0], d_out, uoff[m]);
    if (e != hipSuccess) return hip_status(e, "uncompress");
  }

  // assemble in block order; the first failing block names the status
  Status first = Status::OK();
  out_offsets->resize(n + 1);
  for (size_t i = 0, j = 0; i < n; i++) {
    bool good = true;
    if (types[i] == kNoCompression) {
      out->append(data + offsets[i], offsets[i + 1] - offsets[i]);
    } else if (types[i] == kSnappyCompression) {
      good = len_ok[j] && dec_ok[j];
      if (good) out->append(dec, uoff[j], uoff[j + 1] - uoff[j]);
      j++;
      if (!good && first.ok()) first = Status::Corruption("corrupted compressed block contents");
    } else {
      good = false;
      if (first.ok()) first = Status::Corruption("bad block type");
    }
    if (ok) (*ok)[i] = good ? 1 : 0;
    (*out_offsets)[i + 1] = out->size();
  }
  return first;
}

}  // namespace lsbm
