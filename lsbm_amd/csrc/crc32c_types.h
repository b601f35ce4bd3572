// crc32c_types.h -- layout shared by host (crc32c_engine.cc) and device
// (crc32c_kernels.hip) code: geometry constants, the device table block and
// the ragged-kernel argument block.  Plain C++, no HIP headers.
#pragma once
#include <stdint.h>

// Diagnostic A/B macros that make a build compute wrong results on purpose
// (results not stored, stored CRCs rewritten, bloom probes not set) are
// refused unless the build also says it is a diagnostic one: such a library
// is only ever written under build/ab/ (tools/build_variant.sh), never the
// product lsbm_amd/liblsbm_crc32c.so.
#if (defined(LSBM_DIAG_NO_STORE) || defined(LSBM_DIAG_VERIFY_WRITEBACK) || \
     defined(LSBM_DIAG_NO_PROBE_WRITES)) && !defined(LSBM_DIAG_BUILD)
#error "LSBM_DIAG_* result-changing macros need LSBM_DIAG_BUILD (A/B variant builds only)"
#endif

namespace lsbm {

constexpr int kRowBytes = 128;
constexpr int kGroupLanes = 8;
constexpr int kWaveLanes = 64;
constexpr int kBlockThreads = 1024;
constexpr int kWavesPerWg = kBlockThreads / kWaveLanes;
// The stream kernel (crc32c_stream.hip): 16 waves per CU, 128 VGPRs each
// (A/B, round 3: 16 waves over 12 gain 4-8 points on WAL records).
constexpr int kStreamThreads = 1024;
constexpr int kStreamWavesPerWg = kStreamThreads / kWaveLanes;
constexpr uint32_t kLdsByteTabBytes = 131072;
// Nibble tables (byte offsets into LDS).  Bases are chosen so that an
// and-or can merge the nibble field with the base (disjoint bits).
constexpr uint32_t kNibA4 = 0x20000;     // A^4, 8 x 16 entries (uniform); A^8 and A^12 at
                                         // +512 and +1024 (LSBM_MERGE_PAR: merges in one round trip)
constexpr uint32_t kNibA8 = kNibA4 + 512;
constexpr uint32_t kNibA12 = kNibA4 + 1024;
// A/B (round 5): LSBM_LDS16 holds the A^128 byte tables
// at 16 replicas (64 KiB: lanes l and l + 16 of a half-wave share a bank, a
// 2-way conflict on the row step) and puts byte tables of A^4, laid out the
// same way, in the freed 64 KiB at 0x10000: a merge's three A^4 steps become
// row-step lookups (4 v_perm + 4 ds_read + 2 v_bitop3 each) instead of nibble
// lookups (8 ds_read and ~20 VALU).  Address of (table t, byte b):
//   b << 8 | t << 6 | (lane & 15) << 2   (+ 0x10000 for A^4)
#ifdef LSBM_LDS16
constexpr uint32_t kByteA4 = 0x10000;
#endif
constexpr uint32_t kNibFin = 0x20800;    // A^(116-16li), replicated per lane slot:
                                         // entry (q, nib, lane&31) at q*2048 + nib*128 + lane*4
constexpr uint32_t kRowPowTables = 21;
constexpr uint32_t kNibRowPow = kNibFin + 8 * 16 * 32 * 4;  // A^(128 * 2^i), i = 9..20 (slot i)
// Row shifts of 512 rows and more use slots 9..20; slots 0..8 hold the stream
// kernel's finishing tables: A^(2^i), i = 0..7, and A^-128 (A^e, -128 < e <= 1,
// as A^-128 A^(e + 128), bit by bit).
constexpr uint32_t kRowPowLo = 9;
constexpr uint32_t kNibPow2 = kNibRowPow;              // A^(2^i), i = 0..7: slot i
constexpr uint32_t kNibNeg128 = kNibRowPow + 8 * 512;  // A^-128: slot 8
constexpr uint32_t kNibNeg4 = kNibRowPow + kRowPowTables * 512;  // A^-4 (init injection)
// Stream kernel (crc32c_stream.hip): byte masks of a lane's 16-B chunk and
// the row-start init injections.
constexpr uint32_t kStreamHM = kNibNeg4 + 512;  // KM[lo][hi], 0 <= lo <= hi <= 16: the bytes
                                                // [lo, hi) of a 16-B chunk (4 words, 16-B
                                                // aligned), entry km_entry(lo, hi)
constexpr uint32_t kStreamMasks = 17 * 18 / 2;
// Entry of KM[lo][hi]: the 17 masks [lo, 16) first (the lean rows' only
// lookups, indexed by lo alone), then [lo, hi) for hi < 16 by lo, hi.
constexpr uint32_t km_entry(uint32_t lo, uint32_t hi) {
  return hi >= 16u ? lo : 17u + 16u * lo - ((lo * (lo - 1u)) >> 1) + hi - lo;
}
constexpr uint32_t kStreamR0 = kStreamHM + kStreamMasks * 16;  // R0[d] = A^-d(~0), d = 0..127
constexpr uint32_t kLdsBytes = kStreamR0 + 128 * 4;
constexpr uint32_t kLdsWords = kLdsBytes / 4;
// Besides the image, a kernel's own __shared__ words: the fixed kernel's work
// counter (s_next, crc32c_kernels.hip) -- and the ragged kernels' once they
// take pieces from one.  Reserved here, so that a table added to the image
// fails this assert rather than hipcc's LDS limit on some kernel.
constexpr uint32_t kLdsKernelWords = 20;  // (fixed kernel: s_next and the WgQueue words)

// The cross-XCC work queue's heads (crc32c_units.h): one word per XCC, each
// on its own 64-B line; kQueueWords words of scratch per launch.
#ifndef LSBM_QUEUE_STRIDE  // (A/B builds override)
#define LSBM_QUEUE_STRIDE 16
#endif
constexpr uint32_t kQueueHeads = 8;
constexpr uint32_t kQueueStride = LSBM_QUEUE_STRIDE;
constexpr uint32_t kQueueWords = kQueueHeads * kQueueStride;
static_assert(kLdsBytes % 16 == 0 && kLdsBytes + 4u * kLdsKernelWords <= 160u * 1024u,
              "one LDS image per CU, plus the kernels' work counters");
static_assert(kStreamHM % 16 == 0, "ds_read_b128 of a mask");

constexpr uint32_t kShiftCols = 512;  // unit shifts up to 511 rows (64 KiB frames) by columns
constexpr uint32_t kFinCols = 129;    // A^-z (z < 128) and A^(1 - z) (type-byte extension)

// Tables in device global memory, built once per device by the host (gf2.h).
struct DevConsts {
  uint32_t row_byte[4 * 256];    // byte tables of A^128 (main step)
  uint32_t t0[256];              // A^1 byte table (1-byte extension)
  uint32_t pow_nib[64][128];     // nibble tables of A^(2^k), k = 0..63
  uint32_t neg_nib[128][128];    // nibble tables of A^-z, z = 0..127
  uint32_t neg4_nib[128];        // nibble tables of A^-4
  uint32_t fin_nib[8][128];      // nibble tables of A^(116 - 16 li), li = 0..7 (merge)
  // Column form (col[i] = M(1 << i)) of the matrices the units kernel applies
  // once per unit / per block: an 8-lane group loads one matrix with one 16-B
  // load per lane, issued a round ahead of its use (crc32c_kernels.hip).
  alignas(16) uint32_t shift_cols[kShiftCols][32];  // A^(128 k), k < kShiftCols rows
  alignas(16) uint32_t fin_cols[kFinCols][32];      // A^(e), e = -127 .. 1 (index e + 127)
  // The kernels' LDS image, prebuilt by the host so that each workgroup
  // fills its LDS with ~9 coalesced 16-B loads per thread.
  alignas(16) uint32_t lds_image[kLdsWords];
  alignas(16) uint32_t zero16[4];  // a safe load target for idle lanes
};

// How the ragged kernel finds block i's extent [s, e).
enum ExtentKind : uint32_t {
  kExtOffsets = 0,  // [offsets[i], offsets[i+1])
  kExtHandles = 1,  // [h[2i], h[2i] + h[2i+1])  (BlockHandle {offset, size})
  kExtFixed = 2,    // [i*stride, i*stride + len)
  kExtLogHeaders = 3,  // log record at h = headers[i]: [h + 6, h + 7 + length) where
                       // length = LE16 at h + 4 (common/log_format.h, 7-byte header)
};

// RaggedArgs::flags bits besides the mask bit (1)
constexpr uint32_t kFlagDeferHeaders = 2u;  // kModeLogSeal, stream kernel: out[] first, the headers
                                            // after each wave's last row (out must be set)

enum RaggedMode : uint32_t {
  kModeOut = 0,        // out[i] = crc (masked if flags & 1)
  kModeVerify = 1,     // ok[i] = (crc == expect[i]); mismatches added to *nbad
  kModeSstSeal = 2,    // write trailer [type][Mask(crc(block || type))] after the block;
                       // handles past `limit` (n + 5 bytes must fit) are counted, not written
  kModeSstVerify = 3,  // ok[i] = stored trailer == Mask(crc(block || type)); handles past
                       // `limit` are not ok (ReadBlock's "truncated block read")
  kModeLogSeal = 4,    // header[0..4) = Mask(crc(type || payload)); out[i] too if non-null
  kModeLogVerify = 5,  // ok[i] = Unmask(header[0..4)) == crc(type || payload)
  kModeSstCrc = 6,     // out[i] = Mask(crc(block || type)): the trailer's crc, dense (the
                       // image is not written); handles past `limit` give 0 and are counted
};

// Ragged path: a block's 128-B-aligned frame [row0, row_end) of R rows is cut
// into m = ceil(R / kUnitRows) units of near-equal size (R / m rows, the first
// R % m of them one more).  A unit's raw CRC is shifted to the frame end with
// A^(128 k), k = the frame's rows after the unit; the units of a block are
// summed inside the wave (crc32c_kernels.hip) and the block is finished by the
// lane group holding its last unit.
#ifndef LSBM_CHUNK_BLOCKS  // (A/B builds override; 0 = one contiguous range per wave)
#define LSBM_CHUNK_BLOCKS 128
#endif
// Mean blocks per wave per chunk of the units kernel's chunked sweep, and the
// fewest chunks a batch must make to be swept that way (crc32c_kernels.hip).
constexpr uint32_t kChunkBlocks = LSBM_CHUNK_BLOCKS;
constexpr uint32_t kMinChunks = 8;
constexpr uint32_t kUnitRows = 48;  // A/B 24..96 rows: plateau from 48
constexpr uint32_t kSstUnitRows = 40;  // SSTable trailer modes: a ~4 KiB block is one unit
#ifndef LSBM_SST_PIECE_BLOCKS  // (A/B builds override)
#define LSBM_SST_PIECE_BLOCKS 16
#endif
// SSTable trailer batches: blocks per claimed piece (two 8-block rounds)
constexpr uint32_t kSstPieceBlocks = LSBM_SST_PIECE_BLOCKS;

struct RaggedArgs {
  const uint8_t* base;      // extents are byte offsets from here
  const uint64_t* offsets;  // kExtOffsets
  const uint64_t* handles;  // kExtHandles
  uint64_t stride, len;     // kExtFixed
  uint64_t n;
  const uint32_t* init;  // nullable: per-block init CRC (crc32c::Extend)
  uint32_t* out;
  const uint32_t* expect;
  uint8_t* ok;
  uint32_t* nbad;
  const uint8_t* types;  // kModeSstSeal
  uint8_t* file;         // kModeSstSeal: writable alias of base
  uint32_t flags;
  uint32_t mode;
  uint32_t extents;
  const DevConsts* dc;
  uint32_t u_noinit;     // A^-4(~0): the virtual init bytes when init == nullptr
  uint64_t limit;        // kExtLogHeaders / SST modes: image size; records past it are
                         // empty + bad (~0 = unbounded)
  // Chunked sweep (general Out / Verify batches of >= 8 chunks): wave w's
  // range in chunk c is [bounds[c * nwaves + w], bounds[c * nwaves + w + 1]),
  // c < nchunks, from range_bounds_kernel; null: one range per wave.
  const uint32_t* bounds;
  uint64_t nchunks;
  // Equal-count pieces (no bounds table): piece i is [i q + min(i, r), + q +
  // (i < r)) with q = n / P, r = n % P, P = nchunks * nwaves (set by the host:
  // no 64-bit division on the device).
  uint32_t piece_q, piece_r;
};

}  // namespace lsbm
