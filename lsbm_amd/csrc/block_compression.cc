// block_compression.cc -- include/lsbm/block_compression.h on top of the C
// ABI (include/lsbm_snappy.h).  The blocks are staged to the device once,
// (de)compressed there in one launch, and the results come back whole through
// the pinned bounce; only WriteBlock's keep-or-not rule and the assembly of
// the output run on the host.
#include "../../include/lsbm/block_compression.h"

#include <hip/hip_runtime_api.h>
#include <string.h>

#include "../../include/lsbm_crc32c.h"
#include "../../include/lsbm_snappy.h"
#include "host_stage.h"

namespace lsbm {

namespace {

// Device allocations of one call, freed after the call's stream drains.
struct DeviceScratch {
  std::vector<void*> ptrs;
  PinnedBounce bounce;
  CallStream stream;
  hipError_t alloc(void** p, size_t bytes) {
    const hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~DeviceScratch() {
    if (stream.status() == hipSuccess) (void)hipStreamSynchronize(stream.get());
    for (void* p : ptrs) (void)hipFree(p);
  }
};

Status hip_status(hipError_t e, const char* what) {
  return Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

Status check_offsets(const uint64_t* offsets, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return Status::InvalidArgument("offsets must not decrease");
  return Status::OK();
}

// Makes `device` current; call before a DeviceScratch is made, so that its
// stream belongs to that device.
Status open_device(int device) {
  if (lsbm_crc32c_init(device) != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
  const hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? Status::OK() : hip_status(e, "device");
}

// Rebase offsets[0..n] to start at 0 (the staged copy starts at offsets[0]).
std::vector<uint64_t> rebased(const uint64_t* offsets, size_t n) {
  std::vector<uint64_t> r(n + 1);
  for (size_t i = 0; i <= n; i++) r[i] = offsets[i] - offsets[0];
  return r;
}

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

  s = open_device(device);
  if (!s.ok()) return s;
  DeviceScratch d;
  if (d.stream.status() != hipSuccess) return hip_status(d.stream.status(), "stream");
  const hipStream_t st = d.stream.get();
  void *d_raw = nullptr, *d_off = nullptr, *d_cap = nullptr, *d_comp = nullptr, *d_len = nullptr;
  hipError_t e = d.alloc(&d_raw, total);
  if (e == hipSuccess) e = d.alloc(&d_off, (n + 1) * sizeof(uint64_t));
  if (e == hipSuccess) e = d.alloc(&d_cap, (n + 1) * sizeof(uint64_t));
  if (e == hipSuccess) e = d.alloc(&d_comp, cap[n]);
  if (e == hipSuccess) e = d.alloc(&d_len, n * sizeof(uint64_t));
  if (e == hipSuccess) e = d.bounce.to_device(d_raw, raw + offsets[0], total, st);
  if (e == hipSuccess) e = d.bounce.to_device(d_off, off.data(), (n + 1) * sizeof(uint64_t), st);
  if (e == hipSuccess) e = d.bounce.to_device(d_cap, cap.data(), (n + 1) * sizeof(uint64_t), st);
  if (e != hipSuccess) return hip_status(e, "staging");
  if (lsbm_snappy_compress_dev(d_raw, static_cast<const uint64_t*>(d_off), n, static_cast<uint8_t*>(d_comp),
                               static_cast<const uint64_t*>(d_cap), static_cast<uint64_t*>(d_len),
                               st) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  std::vector<uint64_t> clen(n);
  std::string comp(cap[n], '\0');
  e = d.bounce.to_host(clen.data(), d_len, n * sizeof(uint64_t), st);
  if (e == hipSuccess) e = d.bounce.to_host(&comp[0], d_comp, cap[n], st);
  if (e != hipSuccess) return hip_status(e, "compress");

  // WriteBlock's rule (table/table_builder.cc:187-188), block by block
  types->resize(n);
  out_offsets->resize(n + 1);
  out->reserve(total);
  for (size_t i = 0; i < n; i++) {
    const uint64_t len = off[i + 1] - off[i];
    if (clen[i] != ~0ull && clen[i] < len - len / 8) {
      out->append(comp, cap[i], clen[i]);
      (*types)[i] = kSnappyCompression;
    } else {
      out->append(raw + offsets[i], len);
      (*types)[i] = kNoCompression;
    }
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
    s = open_device(device);
    if (!s.ok()) return s;
    DeviceScratch d;
    if (d.stream.status() != hipSuccess) return hip_status(d.stream.status(), "stream");
    const hipStream_t st = d.stream.get();
    void *d_comp = nullptr, *d_coff = nullptr, *d_ulen = nullptr, *d_ok = nullptr;
    hipError_t e = d.alloc(&d_comp, coff[m]);
    if (e == hipSuccess) e = d.alloc(&d_coff, (m + 1) * sizeof(uint64_t));
    if (e == hipSuccess) e = d.alloc(&d_ulen, m * sizeof(uint64_t));
    if (e == hipSuccess) e = d.alloc(&d_ok, m);
    if (e == hipSuccess) e = d.bounce.to_device(d_comp, packed.data(), coff[m], st);
    if (e == hipSuccess) e = d.bounce.to_device(d_coff, coff.data(), (m + 1) * sizeof(uint64_t), st);
    if (e != hipSuccess) return hip_status(e, "staging");
    // GetUncompressedLength sizes the output windows
    if (lsbm_snappy_uncompressed_length_dev(d_comp, static_cast<const uint64_t*>(d_coff), m,
                                            static_cast<uint64_t*>(d_ulen), static_cast<uint8_t*>(d_ok),
                                            st) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    e = d.bounce.to_host(ulen.data(), d_ulen, m * sizeof(uint64_t), st);
    if (e == hipSuccess) e = d.bounce.to_host(len_ok.data(), d_ok, m, st);
    if (e != hipSuccess) return hip_status(e, "uncompressed length");
    for (size_t j = 0; j < m; j++) uoff[j + 1] = uoff[j] + (len_ok[j] ? ulen[j] : 0);
    void *d_out = nullptr, *d_uoff = nullptr;
    e = d.alloc(&d_out, uoff[m]);
    if (e == hipSuccess) e = d.alloc(&d_uoff, (m + 1) * sizeof(uint64_t));
    if (e == hipSuccess) e = d.bounce.to_device(d_uoff, uoff.data(), (m + 1) * sizeof(uint64_t), st);
    if (e != hipSuccess) return hip_status(e, "staging");
    if (lsbm_snappy_uncompress_dev(d_comp, static_cast<const uint64_t*>(d_coff), m,
                                   static_cast<uint8_t*>(d_out), static_cast<const uint64_t*>(d_uoff),
                                   static_cast<uint8_t*>(d_ok), nullptr, st) != LSBM_OK)
      return Status::IOError(lsbm_crc32c_last_error());
    dec.assign(uoff[m], '\0');
    e = d.bounce.to_host(dec_ok.data(), d_ok, m, st);
    if (e == hipSuccess && uoff[m]) e = d.bounce.to_host(&dec[0], d_out, uoff[m], st);
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
