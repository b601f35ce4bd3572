// table_checksum.cc -- include/lsbm/table_checksum.h on top of the C ABI.
// The file image is staged to the device once, sealed or verified there by
// the ragged kernel in its SSTable modes, and the trailers (seal) or the
// per-block flags (verify) come back.
#include "../../include/lsbm/table_checksum.h"

#include <hip/hip_runtime_api.h>
#include <string.h>

#include "../../include/lsbm_crc32c.h"
#include "host_stage.h"

namespace lsbm {

std::vector<BlockHandle> LayoutBlocks(const std::vector<uint64_t>& sizes, uint64_t* file_size) {
  std::vector<BlockHandle> h(sizes.size());
  uint64_t off = 0;
  for (size_t i = 0; i < sizes.size(); i++) {
    h[i] = BlockHandle{off, sizes[i]};
    off += sizes[i] + kBlockTrailerSize;
  }
  if (file_size) *file_size = off;
  return h;
}

namespace {

struct DeviceBuffers {
  uint8_t* file = nullptr;
  uint64_t* handles = nullptr;
  uint8_t* aux = nullptr;   // types (seal) or ok flags (verify)
  uint32_t* nbad = nullptr;
  PinnedBounce bounce;
  CallStream stream;
  ~DeviceBuffers() {
    if (stream.status() == hipSuccess) (void)hipStreamSynchronize(stream.get());
    if (file) (void)hipFree(file);
    if (handles) (void)hipFree(handles);
    if (aux) (void)hipFree(aux);
    if (nbad) (void)hipFree(nbad);
  }
};

Status hip_status(hipError_t e, const char* what) {
  return Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

Status check_handles(size_t file_size, const BlockHandle* h, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (h[i].offset > file_size || h[i].size > file_size - h[i].offset ||
        file_size - h[i].offset - h[i].size < kBlockTrailerSize)
      return Status::Corruption("truncated block read");  // table/format.cc:88-91
  return Status::OK();
}

// Stage file + handles (+ aux bytes) on `device` (host_stage.h).
Status stage(int device, const void* file, size_t file_size, const BlockHandle* h, size_t n,
             const uint8_t* aux_in, DeviceBuffers* d) {
  int rc = lsbm_crc32c_init(device);
  if (rc != LSBM_OK) return Status::IOError(lsbm_crc32c_last_error());
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = d->stream.status();
  if (e == hipSuccess) e = hipMalloc(&d->file, file_size ? file_size : 1);
  if (e == hipSuccess) e = hipMalloc(&d->handles, n * sizeof(BlockHandle));
  if (e == hipSuccess) e = hipMalloc(&d->aux, n);
  if (e == hipSuccess) e = hipMalloc(&d->nbad, sizeof(uint32_t));
  hipStream_t s = d->stream.get();
  if (e == hipSuccess) e = d->bounce.to_device(d->file, file, file_size, s);
  if (e == hipSuccess) e = d->bounce.to_device(d->handles, h, n * sizeof(BlockHandle), s);  // {offset,size}
  if (e == hipSuccess && aux_in) e = d->bounce.to_device(d->aux, aux_in, n, s);
  if (e == hipSuccess) e = hipMemsetAsync(d->nbad, 0, sizeof(uint32_t), s);
  return e == hipSuccess ? Status::OK() : hip_status(e, "staging");
}

}  // namespace

Status SealBlocks(int device, char* file, size_t file_size, const BlockHandle* handles,
                  const uint8_t* types, size_t n) {
  if (n == 0) return Status::OK();
  if (!file || !handles || !types) return Status::InvalidArgument("null pointer");
  Status s = check_handles(file_size, handles, n);
  if (!s.ok()) return s;
  DeviceBuffers d;
  s = stage(device, file, file_size, handles, n, types, &d);
  if (!s.ok()) return s;
  if (lsbm_sst_seal_dev(d.file, file_size, d.handles, d.aux, n, nullptr, d.stream.get()) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  // Bring the image back whole through the pinned bounce: one streamed copy
  // instead of one 5-byte hipMemcpyAsync (a runtime call) per block.  The
  // device image is the host image plus the trailers.
  const hipError_t e = d.bounce.to_host(file, d.file, file_size, d.stream.get());
  if (e != hipSuccess) return hip_status(e, "seal");
  return Status::OK();
}

Status VerifyBlocks(int device, const char* file, size_t file_size, const BlockHandle* handles,
                    size_t n, std::vector<uint8_t>* ok) {
  if (ok) ok->assign(n, 1);
  if (n == 0) return Status::OK();
  if (!file || !handles) return Status::InvalidArgument("null pointer");
  Status s = check_handles(file_size, handles, n);
  if (!s.ok()) return s;
  DeviceBuffers d;
  s = stage(device, file, file_size, handles, n, nullptr, &d);
  if (!s.ok()) return s;
  if (lsbm_sst_verify_dev(d.file, file_size, d.handles, n, d.aux, d.nbad, d.stream.get()) != LSBM_OK)
    return Status::IOError(lsbm_crc32c_last_error());
  uint32_t nbad = 0;
  hipError_t e = d.bounce.to_host(&nbad, d.nbad, sizeof(nbad), d.stream.get());
  if (e == hipSuccess && ok) e = d.bounce.to_host(ok->data(), d.aux, n, d.stream.get());
  if (e != hipSuccess) return hip_status(e, "verify");
  return nbad ? Status::Corruption("block checksum mismatch") : Status::OK();
}

}  // namespace lsbm
