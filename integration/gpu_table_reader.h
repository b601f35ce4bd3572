// integration/gpu_table_reader.h -- the compaction read side: every data
// block of an input table verified by ONE lsbm::VerifyBlocks call on the GPU,
// then the table iterated from memory with no per-block CRC.
//
// What the reference does: DoCompactionWork iterates its input tables with
// ReadOptions::verify_checksums = paranoid_checks (lsbm/version_set.cc:2311);
// with it on, every data block goes through ReadBlock's check -- pread into
// `new char[n + 5]`, then crc32c::Value(data, n + 1) against the stored
// trailer on the CPU, block by block (table/format.cc:66-103).  A compaction
// reads each input table whole, front to back.
//
// What this does instead (OpenVerifiedTable): one read of the whole file into
// a heap image (owned by the TableImageFile the table reads from), the index block parsed with the reference's own ReadBlock and
// Block (no checksum, as Table::Open reads it, table/table.cc:67-76), ONE
// VerifyBlocks call over all data blocks -- the image is writable heap memory,
// so it is page-locked for the call and DMA-ed in place (~0.35 ms per 16 MiB
// on an MI355X) -- and then the reference's Table::Open over an in-memory
// RandomAccessFile of the image (reads are pointers into it: no copy, no
// syscall), to be iterated with verify_checksums = false.  Entries are the
// same as the reference's verified iteration.  A mismatch returns the
// status ReadBlock would ("Corruption: block checksum mismatch", or
// "Corruption: truncated block read" for a handle past the file), and the
// caller can fall back to the reference's own verified iteration, which then
// reproduces its exact behaviour around the bad block (it skips the block and
// keeps the first error, table/two_level_iterator.cc).  A verify the device
// cannot do (a status other than Corruption: no device, a HIP error, no
// staging memory) is done on the CPU with the library's scalar crc32c
// (integration/gpu_fallback.h), with the same statuses: a GPU problem never
// fails the read.
//
// Tested against the reference's reader in tests/cpp/ref_table_builder_gpu.cc
// (oracle/Makefile `gputable`, run on the GPU by tests/test_gpu_parity.py).
#ifndef LSBM_INTEGRATION_GPU_TABLE_READER_H_
#define LSBM_INTEGRATION_GPU_TABLE_READER_H_

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "integration/gpu_fallback.h"
#include "integration/image_pool.h"
#include "leveldb/env.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "lsbm/table_checksum.h"
#include "table/block.h"
#include "table/format.h"

namespace leveldb {

// A table image held in memory as a RandomAccessFile, owning the image:
// reads return pointers into it (ReadBlock then uses them in place,
// table/format.cc:105-112).  The buffer is `new char[]` (no zero fill: the
// file's bytes are read straight into it), writable heap memory, so
// VerifyBlocks page-locks it for its call; or a pooled image, page-locked
// already once it has been used.
class TableImageFile : public RandomAccessFile {
 public:
  explicit TableImageFile(uint64_t size) : own_(new char[size ? size : 1]), data_(own_), size_(size) {}
  // An image from `pool` (integration/image_pool.h), back to it with this
  // file: its pages stay faulted in and page-locked from table to table.
  TableImageFile(uint64_t size, ImagePool* pool) : pool_(pool), pooled_(pool->Take(size ? size : 1)), size_(size) {
    std::string& b = pooled_->bytes;
    if (b.size() < size) b.resize(size);  // (within its capacity: the image does not move)
    data_ = &b[0];
  }
  ~TableImageFile() {
    if (pooled_) pool_->Give(pooled_);
    delete[] own_;
  }
  Status Read(uint64_t offset, size_t n, Slice* result, char*) const {
    if (offset > size_) return Status::IOError("table image", "read past the end");
    *result = Slice(data_ + offset, std::min<uint64_t>(n, size_ - offset));
    return Status::OK();
  }
  char* data() { return data_; }
  uint64_t size() const { return size_; }

 private:
  char* own_ = nullptr;
  ImagePool* pool_ = nullptr;
  PooledImage* pooled_ = nullptr;
  char* data_;
  uint64_t size_;
  TableImageFile(const TableImageFile&);
  void operator=(const TableImageFile&);
};

// Reads `file` (size bytes) whole into a new *image_file, verifies every data
// block on HIP device `device` in one call, and on success opens *table over
// it (the caller deletes the table, then the image file).  *data_blocks
// receives the number of blocks verified.
// pool (optional): the image comes from it (integration/image_pool.h) and
// goes back when *image_file is deleted.
inline Status OpenVerifiedTable(const Options& options, uint64_t file_number, RandomAccessFile* file,
                                uint64_t size, int device, TableImageFile** image_file, Table** table,
                                size_t* data_blocks, ImagePool* pool = nullptr) {
  *table = nullptr;
  *image_file = nullptr;
  *data_blocks = 0;
  if (size < Footer::kEncodedLength) return Status::InvalidArgument("file is too short to be an sstable");
  TableImageFile* f = pool ? new TableImageFile(size, pool) : new TableImageFile(size);
  Slice got;
  Status s = file->Read(0, size, &got, f->data());
  if (s.ok() && got.size() != size) s = Status::Corruption("truncated block read");
  if (!s.ok()) {
    delete f;
    return s;
  }
  if (got.data() != f->data()) memcpy(f->data(), got.data(), size);  // (a file that hands out its own memory)
  Slice tail(f->data() + size - Footer::kEncodedLength, Footer::kEncodedLength);
  Footer footer;
  s = footer.DecodeFrom(&tail);

  // the data blocks, from the index block (read as Table::Open reads it)
  BlockContents index_contents;
  if (s.ok()) s = ReadBlock(f, ReadOptions(), footer.index_handle(), &index_contents);
  std::vector<lsbm::BlockHandle> handles;
  if (s.ok()) {
    Block index(index_contents);
    Iterator* it = index.NewIterator(options.comparator);
    for (it->SeekToFirst(); it->Valid() && s.ok(); it->Next()) {
      Slice v = it->value();
      BlockHandle h;
      s = h.DecodeFrom(&v);
      if (s.ok()) handles.push_back(lsbm::BlockHandle{h.offset(), h.size()});
    }
    if (s.ok()) s = it->status();
    delete it;
  }

  // ONE check of every data block's trailer on the GPU (ReadBlock's
  // verify_checksums test, table/format.cc:95-103, for all of them at once)
  if (s.ok()) {
    const lsbm::Status v = lsbm::VerifyBlocks(device, f->data(), size, handles.data(), handles.size(), nullptr,
                                                lsbm::kImagesWritable);
    if (v.IsCorruption()) {
      const std::string m = v.ToString();
      const std::string kC = "Corruption: ";
      s = Status::Corruption(m.substr(m.compare(0, kC.size(), kC) == 0 ? kC.size() : 0));
    } else if (!v.ok()) {
      // the device could not check them (no device, a HIP error, no staging
      // memory): ReadBlock's check on the CPU instead, same statuses
      // (integration/gpu_fallback.h), so a GPU problem never fails a read
      s = VerifyBlocksOnHost(f->data(), size, handles.data(), handles.size());
      GpuFallbacks().verifies.fetch_add(1, std::memory_order_relaxed);
    }
  }
  if (s.ok()) s = Table::Open(options, file_number, f, size, table);
  if (!s.ok()) {
    delete f;
    return s;
  }
  *data_blocks = handles.size();
  *image_file = f;
  return Status::OK();
}

}  // namespace leveldb

#endif  // LSBM_INTEGRATION_GPU_TABLE_READER_H_
