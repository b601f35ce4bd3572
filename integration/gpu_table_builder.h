// integration/gpu_table_builder.h -- the reference's TableBuilder with every
// block trailer sealed on the GPU, ONE lsbm::SealBlocks call per table.
//
// What the reference does per block (table/table_builder.cc:237-255,
// WriteRawBlock): Append(block), then crc32c::Value + Extend(type) + Mask on
// the CPU, then Append(trailer).  Finish (:261-316) writes the filter,
// metaindex and index blocks the same way, then the footer.
//
// What this builder does instead: the table image grows in memory; each
// block's bytes are appended and its 5 trailer bytes RESERVED (its handle and
// CompressionType recorded); at Finish, after the index block, one
// SealBlocks call (include/lsbm/table_checksum.h) fills every trailer --
// data, filter, metaindex and index blocks -- on the GPU, the footer is
// appended and the finished image goes to the WritableFile in one Append.
// A seal the device cannot do (any non-OK SealBlocks status) is done on the
// CPU with the library's scalar crc32c (integration/gpu_fallback.h): the
// reference's checksum never fails, so neither does this builder's, and the
// file is the same bytes either way.
// The image is heap memory (std::string), so the call page-locks it for its
// duration and DMAs it in place: ~0.36 ms per 16 MiB table on an MI355X
// against ~8.7 ms of one core for the reference's per-block Extend loop
// (DESIGN.md section 5).
//
// Everything else is the reference's own code: BlockBuilder
// (table/block_builder.cc), FilterBlockBuilder (table/filter_block.cc),
// BlockHandle / Footer encodings (table/format.cc), the comparator's
// separators, port::Snappy_Compress and the 12.5% rule (table_builder.cc:
// 181-193).  The output is byte-identical to TableBuilder's for the same
// Options and key stream (tests/cpp/ref_table_builder_gpu.cc, run on the GPU
// by tests/test_gpu_parity.py).  Not carried over: lsbm's pre_caching
// (inserting just-written blocks into the block cache, :196-230), which does
// not touch the file bytes; the patch in INTEGRATION.md keeps it in place.
//
// Written against the reference's headers (compiled with them by
// oracle/Makefile `gputable`); a maintainer would fold it into TableBuilder
// itself ("TableBuilder").
#ifndef LSBM_INTEGRATION_GPU_TABLE_BUILDER_H_
#define LSBM_INTEGRATION_GPU_TABLE_BUILDER_H_

#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "leveldb/comparator.h"
#include "leveldb/env.h"
#include "leveldb/filter_policy.h"
#include "leveldb/options.h"
#include "integration/gpu_fallback.h"
#include "lsbm/table_checksum.h"
#include "port/port.h"
#include "table/block_builder.h"
#include "table/filter_block.h"
#include "table/format.h"

namespace leveldb {

class GpuTableBuilder {
 public:
  // Builds a table for `file` (not closed here), sealing on HIP `device`.
  // size_hint: the table size the caller expects (a compaction knows its
  // MaxOutputFileSize): the image is reserved once instead of growing by
  // reallocation, each of which copies everything so far.
  // image: where the table image is built (cleared here; its capacity kept),
  // so that a caller can hand the same buffer to table after table: its pages
  // are then faulted in once, and may stay page-locked (table_builder_gpu.cc);
  // null: a buffer of the builder's own.
  // move / move_arg: the image-move observer (SetImageMoveObserver), in
  // force from the constructor's own reserve on: a caller that page-locked
  // `image` is told before any reallocation, this one included.
  typedef void (*ImageMoveObserver)(void* arg);
  GpuTableBuilder(const Options& options, WritableFile* file, int device = 0, uint64_t size_hint = 0,
                  std::string* image = nullptr, ImageMoveObserver move = nullptr, void* move_arg = nullptr)
      : image_(image ? *image : own_image_),
        move_observer_(move),
        move_arg_(move_arg),
        options_(options),
        index_options_(options),
        file_(file),
        device_(device),
        data_(&options_),
        index_(&index_options_),
        filter_(options.filter_policy ? new FilterBlockBuilder(options.filter_policy) : nullptr) {
    index_options_.block_restart_interval = 1;  // (every index entry a restart point)
    if (filter_) filter_->StartBlock(0);
    image_.clear();
    const size_t want = ImageBytesFor(size_hint);
    if (want > image_.capacity()) {  // (never smaller: reserve may shrink)
      if (move_observer_) move_observer_(move_arg_);
      image_.reserve(want);
    }
  }
  ~GpuTableBuilder() { delete filter_; }

  // the image capacity reserved for a table of about size_hint bytes (+ the
  // meta blocks and the last block)
  static size_t ImageBytesFor(uint64_t size_hint) {
    return size_hint ? size_hint + size_hint / 8 + (64u << 10) : 0;
  }

  // TableBuilder::Add: keys in comparator order.
  void Add(const Slice& key, const Slice& value) {
    if (closed_ || !status_.ok()) return;
    if (index_due_) {
      // the previous data block's index key: a short separator between its
      // last key and this one
      options_.comparator->FindShortestSeparator(&last_key_, key);
      AddIndexEntry();
    }
    if (filter_) filter_->AddKey(key);
    last_key_.assign(key.data(), key.size());
    entries_++;
    data_.Add(key, value);
    if (data_.CurrentSizeEstimate() >= options_.block_size) Flush();
  }

  // TableBuilder::ChangeOptions (table/table_builder.cc:92-106): the
  // comparator may not change; the block builders see the new options.
  Status ChangeOptions(const Options& options) {
    if (options.comparator != options_.comparator)
      return Status::InvalidArgument("changing comparator while building table");
    options_ = options;
    index_options_ = options;
    index_options_.block_restart_interval = 1;
    return Status::OK();
  }

  // An observer of each data block as it is placed (its contents as stored,
  // i.e. after compression), for what the reference does beside the write:
  // lsbm's pre-caching (table/table_builder.cc:195-230).  `closing` is true
  // for the block Finish closes, which the reference never caches (it calls
  // Flush(false), :263).
  typedef void (*DataBlockObserver)(void* arg, const Slice& contents, bool closing);
  void SetDataBlockObserver(DataBlockObserver fn, void* arg) {
    observer_ = fn;
    observer_arg_ = arg;
  }

  // Called before the image buffer reallocates (it is about to move): a
  // caller that page-locked the buffer unlocks it here.
  void SetImageMoveObserver(ImageMoveObserver fn, void* arg) {
    move_observer_ = fn;
    move_arg_ = arg;
  }

  // Closes the current data block (its trailer reserved, not computed).
  void Flush() {
    if (closed_ || !status_.ok() || data_.empty()) return;
    PlaceBlock(&data_, &due_handle_, true);
    index_due_ = true;
    if (filter_) filter_->StartBlock(image_.size());
  }

  // The meta blocks, ONE seal of every trailer on the GPU, the footer, and
  // the whole image into the file.
  Status Finish() {
    closing_ = true;
    Flush();
    closed_ = true;
    BlockHandle filter_at, meta_at, index_at;
    if (status_.ok() && filter_) Place(filter_->Finish(), kNoCompression, &filter_at);
    if (status_.ok()) {
      BlockBuilder meta(&options_);
      if (filter_) {
        std::string where;
        filter_at.EncodeTo(&where);
        meta.Add(std::string("filter.") + options_.filter_policy->Name(), where);
      }
      PlaceBlock(&meta, &meta_at);
    }
    if (status_.ok()) {
      if (index_due_) {
        options_.comparator->FindShortSuccessor(&last_key_);
        AddIndexEntry();
      }
      PlaceBlock(&index_, &index_at);
    }
    if (status_.ok()) {
      seal_calls_++;
      const lsbm::Status s =
          lsbm::SealBlocks(device_, &image_[0], image_.size(), handles_.data(), types_.data(), handles_.size());
      if (!s.ok()) {
        // The reference's checksum cannot fail (WriteRawBlock, table/
        // table_builder.cc:243-250), and a failed compaction stops lsbm's
        // writes (bg_error_, lsbm/db_impl.cc:567-573): a device that cannot
        // seal (no device, a HIP error, no staging memory) costs the CPU
        // trailers instead, the same bytes (integration/gpu_fallback.h).
        // The handles are the builder's own, all inside the image, so the
        // seal cannot have refused them.
        SealTrailersOnHost(&image_[0], handles_.data(), types_.data(), handles_.size());
        host_seals_++;
        GpuFallbacks().seals.fetch_add(1, std::memory_order_relaxed);
        last_gpu_error_ = s.ToString();
      }
    }
    if (status_.ok()) {
      Footer footer;
      footer.set_metaindex_handle(meta_at);
      footer.set_index_handle(index_at);
      std::string tail;
      footer.EncodeTo(&tail);
      Room(tail.size());
      image_.append(tail);
      status_ = file_->Append(image_);
    }
    return status_;
  }

  void Abandon() { closed_ = true; }
  Status status() const { return status_; }
  uint64_t NumEntries() const { return entries_; }
  uint64_t FileSize() const { return image_.size(); }  // (reserved trailers included, as the reference's offset)
  size_t SealCalls() const { return seal_calls_; }
  // Finish calls whose seal fell back to the CPU, and the GPU's status then
  size_t HostSeals() const { return host_seals_; }
  const std::string& LastGpuError() const { return last_gpu_error_; }
  size_t Blocks() const { return handles_.size(); }
  // every block placed so far: data blocks, then filter, metaindex, index
  const std::vector<lsbm::BlockHandle>& Handles() const { return handles_; }

 private:
  // Capacity for `more` bytes; a reallocation (doubling) is announced first.
  void Room(size_t more) {
    if (image_.size() + more <= image_.capacity()) return;
    if (move_observer_) move_observer_(move_arg_);
    image_.reserve(std::max(2 * image_.capacity(), image_.size() + more));
  }

  void AddIndexEntry() {
    std::string where;
    due_handle_.EncodeTo(&where);
    index_.Add(last_key_, where);
    index_due_ = false;
  }

  // A built block: compressed when the options ask for it and snappy saves
  // at least 1/8 (table/table_builder.cc:176-193), else raw.
  void PlaceBlock(BlockBuilder* b, BlockHandle* at, bool data_block = false) {
    const Slice raw = b->Finish();
    Slice contents = raw;
    CompressionType type = kNoCompression;
    if (options_.compression == kSnappyCompression &&
        port::Snappy_Compress(raw.data(), raw.size(), &packed_) && packed_.size() < raw.size() - raw.size() / 8u) {
      contents = packed_;
      type = kSnappyCompression;
    }
    if (data_block && observer_) observer_(observer_arg_, contents, closing_);
    Place(contents, type, at);
    packed_.clear();
    b->Reset();
  }

  // The block's bytes, then kBlockTrailerSize bytes the seal fills in.
  void Place(const Slice& contents, CompressionType type, BlockHandle* at) {
    at->set_offset(image_.size());
    at->set_size(contents.size());
    handles_.push_back(lsbm::BlockHandle{image_.size(), contents.size()});
    types_.push_back(static_cast<uint8_t>(type));
    Room(contents.size() + kBlockTrailerSize);
    image_.append(contents.data(), contents.size());
    image_.append(kBlockTrailerSize, '\0');
  }

  std::string own_image_;
  std::string& image_;  // the table so far: blocks with reserved trailers
  ImageMoveObserver move_observer_ = nullptr;
  void* move_arg_ = nullptr;
  Options options_;
  Options index_options_;
  WritableFile* file_;
  int device_;
  Status status_;
  BlockBuilder data_;
  BlockBuilder index_;
  FilterBlockBuilder* filter_;
  std::string last_key_;
  uint64_t entries_ = 0;
  bool index_due_ = false;  // a data block was closed and its index entry waits for the next key
  bool closed_ = false;
  BlockHandle due_handle_;
  std::string packed_;
  std::vector<lsbm::BlockHandle> handles_;  // every block of the image, for the seal
  std::vector<uint8_t> types_;
  size_t seal_calls_ = 0;
  size_t host_seals_ = 0;
  std::string last_gpu_error_;
  bool closing_ = false;  // inside Finish
  DataBlockObserver observer_ = nullptr;
  void* observer_arg_ = nullptr;

  GpuTableBuilder(const GpuTableBuilder&);
  void operator=(const GpuTableBuilder&);
};

}  // namespace leveldb

#endif  // LSBM_INTEGRATION_GPU_TABLE_BUILDER_H_
