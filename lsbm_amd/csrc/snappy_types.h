// snappy_types.h -- argument blocks shared by snappy_engine.cc (host) and
// snappy_kernels.hip (device).  Plain C++, no HIP headers.
#pragma once
#include <stdint.h>

namespace lsbm {

// One wave per block, one wave per workgroup.  A block whose working set fits
// the wave's LDS slice is decoded / encoded in LDS in a first pass; a larger
// one is left to a second pass with larger slices, or against global memory
// (the decoder's output; the encoder's fragment bytes, its table staying in
// LDS).
constexpr uint32_t kSnapThreads = 64;
// decoder slices hold the output window (the compressed bytes are read from
// global memory): pass 1 uses small slices (more waves in flight), pass 2
// large ones.  5 KiB: a db_bench block (4,117-4,122 B) fits, 32 waves per CU
// (the hardware's maximum).  (Round 2's decoder staged the compressed bytes
// in the slice too: 7 KiB, 22 waves per CU; A/B 8 / 7 / 6.5 KiB 171 / 189 /
// 187 GB/s.  A/B builds with LSBM_SNAP_STAGED_INPUT still do.)
#ifndef LSBM_SNAP_DEC_LDS  // (A/B builds override)
#ifdef LSBM_SNAP_STAGED_INPUT
#define LSBM_SNAP_DEC_LDS 7168
#else
#define LSBM_SNAP_DEC_LDS 5120
#endif
#endif
constexpr uint32_t kSnapDecLds = LSBM_SNAP_DEC_LDS;
// the deferred passes' slices (output window only): for blocks of the 8, 16,
// 32 and 64 KiB block sizes (which run a little over)
constexpr uint32_t kSnapDecTierLds[4] = {9216, 17408, 33792, 81920};
constexpr int kSnapDecTiers = 4;
constexpr uint32_t kSnapDecScan = 16;  // blocks per ballot scan in the deferred passes, decoder and encoder (<= 64)
// encoder: hash table (2 B/entry) + fragment bytes in a 22 KiB slice (a
// 4 KiB block with its 8,192-entry table needs 20.1 KiB), then the match
// search's hash-bucket counters (one byte each): 22.5 KiB, 7 waves per CU
constexpr uint32_t kSnapEncSlice = 22528;
constexpr uint32_t kSnapEncBuckets = 512;
constexpr uint32_t kSnapEncLds = kSnapEncSlice + kSnapEncBuckets;
// the encoder's middle pass: 48 KiB per wave (a 2^14-entry table and up to
// ~16 KiB of fragment), 3 waves per CU
constexpr uint32_t kSnapEncMidLds = 48 * 1024;
constexpr uint32_t kSnapEncMidSlice = kSnapEncMidLds - kSnapEncBuckets;
#ifndef LSBM_SNAP_PROBES
#define LSBM_SNAP_PROBES 24
#endif
constexpr uint32_t kSnapProbes = LSBM_SNAP_PROBES;  // match-search probes per wave step (<= 64)
constexpr uint32_t kSnapMaxTableBits = 15;             // libsnappy >= 1.1.10 (oracle/snappy_oracle.c)
constexpr uint32_t kSnapMaxTable = 1u << kSnapMaxTableBits;
constexpr uint32_t kSnapFragment = 65536;              // snappy kBlockSize
constexpr uint32_t kSnapDecWgsPerCu = 160 * 1024 / kSnapDecLds;  // LDS-limited residency

constexpr uint32_t kSnapEncWgsPerCu = 160 * 1024 / kSnapEncLds;
// encoder pass 2 (blocks that pass 1 cannot hold): the largest hash table in
// LDS (2^15 entries), fragment bytes from global memory; 2 waves per CU
constexpr uint32_t kSnapEncLargeLds = 2 * kSnapMaxTable + kSnapEncBuckets;
constexpr uint32_t kSnapEncLargeWgsPerCu = 160 * 1024 / kSnapEncLargeLds;
constexpr uint32_t kSnapEncMidWgsPerCu = 160 * 1024 / kSnapEncMidLds;
constexpr uint64_t kSnapDeferred = ~0ull - 1;  // out_len of a block left for pass 2

struct SnapLenArgs {
  const uint8_t* base;
  const uint64_t* offsets;  // block i = base[offsets[i], offsets[i+1])
  uint64_t* ulen;           // GetUncompressedLength result (0 on failure)
  uint8_t* ok;
  uint64_t n;
};

struct SnapDecArgs {
  const uint8_t* base;
  const uint64_t* offsets;      // compressed block i = base[offsets[i], offsets[i+1])
  uint8_t* out;
  const uint64_t* out_offsets;  // output i = out[out_offsets[i], out_offsets[i+1]) (capacity)
  uint8_t* ok;
  uint32_t* n_bad;              // nullable
  uint64_t n;
};

struct SnapEncArgs {
  const uint8_t* base;
  const uint64_t* offsets;      // raw block i = base[offsets[i], offsets[i+1])
  uint8_t* out;
  const uint64_t* out_offsets;  // compressed i starts at out + out_offsets[i]
  uint64_t* out_len;            // compressed size (UINT64_MAX: block >= 2^32 bytes)
  uint64_t n;
};

}  // namespace lsbm
