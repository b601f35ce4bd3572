// crc32c_stream.hip -- the stream-major CRC-32C kernel for densely packed
// images: SSTable files, WAL / MANIFEST log images, offsets[] batches.
//
// The units kernel (crc32c_units.h) gives each 8-lane group one unit of one
// block per round and runs the round in lock-step for as many rows as its
// longest unit.  On short or uneven blocks most of its loads read the zero
// pad (343 B of 1,024 B per wave-load on WAL records, 691 B on config 4) and
// the round overhead is paid per ~10 rows.  Here the rows of the image are
// streamed regardless of block boundaries:
//
//   * a wave takes a piece of consecutive blocks (as the units kernel) and
//     cuts it into sub-pieces of at most 63 blocks, whose extents it loads
//     into registers (one per lane) and checks: ascending and non-overlapping
//     (s_j >= e_{j-1}), within a 2 GiB window; a sub-piece ends before the
//     first block that is not.  When that leaves fewer than 16 blocks (blocks
//     out of order), or a block alone spans 2 GiB, the units walk (any order,
//     any size), inlined after the stream loop, takes the rest of the wave's
//     range from that block on.  (Round 3 called it out of line and redid the
//     wave's whole range: out-of-order headers ran at 33% of HBM peak against
//     the units kernel's 43-54%; the out-of-line walk spills in its rounds.
//     Round 4's first try, the out-of-line walk per 63-block window, ran at
//     26-30%.)
//   * the sub-piece's rows [floor(s_first / 128), last row] are cut into 8
//     segments of Q rows, one per lane group, and every group streams its
//     segment row after row with the fixed kernel's access pattern: one 16-B
//     load per lane per 128-B row through a buffer descriptor bounded to the
//     sub-piece (chunks outside it read zeros), the braids c_m = A^128(c_m)
//     ^ w_m (util/crc32c.cc:295-302 for a 128-B stride);
//   * every row is the plain row step; a row where some group starts or ends
//     a block is then fixed up, as selects every group runs (a group-uniform
//     branch here cost ~100 instructions and three dependent LDS round trips
//     per such row, and on WAL records most rows are such rows): the ending
//     block's braids through its end (a 16-B byte mask) are saved into the
//     group's slot, the starting block's braids become its bytes of the row
//     with its init register ~0 injected as A^-(s mod 128)(~0) (an LDS table),
//     so that the register is exactly ~0 when its first byte is absorbed
//     (:289).  The masks, the init word and the pointers' next values are read
//     when the previous event was handled.  A row where a group starts and
//     ends the same block goes through a general fix-up loop;
//   * when a group must save an end while its slot is full, every group's
//     oldest saved end is merged (merge_braids, one call for all 8 groups) and
//     each raw CRC goes to the lane of its block (block j of the sub-piece:
//     lane j) by one ds_bpermute from the group where it ends;
//   * at the sub-piece end every lane finishes its own block: A^-z (z = the
//     bytes after e in its last row) from the LDS power tables, the mode
//     (CRC, masked CRC, verify, SSTable trailer CRC / check, log header seal /
//     check) against the stored value it loaded when the sub-piece began,
//     and one coalesced store per wave (no global load or store in the row
//     loop besides the rows);
//   * a block that crosses into the next group's segment leaves its braids
//     there at the segment end (T); the group where it ends saves the rest
//     (its head).  At the sub-piece end T pieces are merged, shifted to the
//     block's last row by A^(128 k), summed per block by a segmented xor-scan
//     over the groups and added to the head before it is finished.
//
// Every row is read once per wave and fully used: no pad loads, no per-round
// lock-step.  Results are those of crc32c::Extend(~0-init) over each block
// (util/crc32c.cc:286-329), exactly as the units kernel computes them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_units.h"

namespace lsbm {

#ifdef LSBM_STREAM_STATS
// diagnostic counters (tools/stream_stats.sh): wave-rows, slow wave-rows,
// general half-steps, general iterations, flushes, slot merges, sub-pieces,
// group events
// and wave cycles in: sub-piece setup, row loop, flushes, general rows, (4: unused),
// sub-piece tail, the tail's per-lane finish (part of the tail)
__device__ unsigned long long g_stream_stats[16];
#define LSBM_STAT(i, v) (st[i] += (v))
#define LSBM_TIC(i) const uint64_t tic_##i = __builtin_readcyclecounter()
#define LSBM_TOC(i) (tm[i] += __builtin_readcyclecounter() - tic_##i)
#else
#define LSBM_STAT(i, v) ((void)0)
#define LSBM_TIC(i) ((void)0)
#define LSBM_TOC(i) ((void)0)
#endif

constexpr uint32_t kSubBlocks = 63;   // blocks per sub-piece: one extent per lane; lane 63 always
                                      // holds the sentinel block that never starts or ends
#ifndef LSBM_STREAM_PREISSUE  // (A/B builds: 1 = issue the next sub-piece's first rows before the tail; measured -4.5 points on config 4, no gain on WAL: off)
#define LSBM_STREAM_PREISSUE 0
#endif
#ifndef LSBM_STREAM_MERGE2  // (A/B builds: 0 = the tail flushes, then merges the open block)
#define LSBM_STREAM_MERGE2 1
#endif
#ifndef LSBM_STREAM_EARLY_BANKS  // (A/B builds: 0 = a segment's first banks issued after the setup's picks)
#define LSBM_STREAM_EARLY_BANKS 1
#endif
#ifndef LSBM_STREAM_SLOTS  // (A/B builds override: 1 or 2)
#define LSBM_STREAM_SLOTS 1
#endif
constexpr uint32_t kSlots = LSBM_STREAM_SLOTS;  // block ends saved per group between flushes
static_assert(kSlots == 1 || kSlots == 2, "one or two slots");
constexpr int kStreamAux = 2;         // buffer-load policy: non-temporal (read once)
constexpr uint32_t kBank = 3;         // rows per load bank (two in flight); round-2 A/B on the
                                      // fixed kernel: 3-6 rows per bank alike

typedef const __attribute__((address_space(1), aligned(1))) uint32_t* gptr_u32u;

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, uint32_t d) {
  return (uint64_t)(uint32_t)__shfl_up((int)(uint32_t)v, d) |
         ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d) << 32);
}
// Last row of block [s, e) (relative byte offsets): the row of byte e - 1, or
// of s for an empty block.
__device__ __forceinline__ uint32_t end_row(uint32_t s, uint32_t e) {
  return e > s ? (e - 1u) >> 7 : s >> 7;
}

template <uint32_t kR, uint32_t kMode, uint32_t kExt>
__global__ __launch_bounds__(kStreamThreads) void crc32c_stream_kernel(RaggedArgs args) {
  static_assert(kR % 8 == 0 && kR <= 32, "rows per step: banks of 4");
  args.mode = kMode;
  args.extents = kExt;
  constexpr bool kSstModes = kMode == kModeSstVerify || kMode == kModeSstCrc;
  constexpr uint32_t kFallbackRows = kSstModes ? kSstUnitRows : LSBM_UNIT_ROWS;
  const DevConsts* __restrict__ dc = args.dc;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 3, li = lane & 7u;
  const uint32_t lb = row_lane_base(lane);
  const uint32_t L0 = lb | kRowTab[0], L1 = lb | kRowTab[1], L2 = lb | kRowTab[2], L3 = lb | kRowTab[3];
  const uint32_t lane_fin = kNibFin | lb;
  const uint64_t wave = (uint64_t)blockIdx.x * kStreamWavesPerWg +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kStreamWavesPerWg;
  bool chunked;
  uint32_t pi, p_end;
  uint64_t b_lo, b_hi;
  DIAG_STAMP_W(0, wave);
  wave_range<kMode, kExt>(args, wave, nwaves, chunked, pi, p_end, b_lo, b_hi);
  if (chunked) piece_range(args, pi, p_end, b_lo, b_hi);
  // a chunked sweep's later pieces are claimed from an LDS counter
  // (next_piece, crc32c_units.h), also by the units walk it may fall back to
  __shared__ uint32_t s_claim;
  lds_u32* claim = nullptr;
#ifndef LSBM_PIECES_STATIC
  if (chunked) claim = (lds_u32*)&s_claim;
  if (threadIdx.x == 0) s_claim = kStreamWavesPerWg;  // (ordered by load_lds_tables' barrier)
#endif
  load_lds_tables<kStreamThreads>(g_lds, dc);
  DIAG_STAMP_W(1, wave);
  const uint64_t base = reinterpret_cast<uint64_t>(args.base);
  const uint64_t dummy = reinterpret_cast<uint64_t>(dc->zero16);
  const char* lds_c = reinterpret_cast<const char*>(g_lds);

  uint32_t nbad = 0;  // bad blocks (wave-uniform)

#ifdef LSBM_STREAM_STATS
  uint32_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  // the first block the stream leaves to the units walk (~0: none; wave-uniform)
  uint64_t resume = ~0ull;
  // The next sub-piece's extents are loaded while this one streams (its log
  // record lengths, loads that depend on them, behind its first rows): a
  // sub-piece starts without waiting for them.
  ExtRaw nx = {0, 0};
  uint64_t nx_b = ~0ull;  // nx holds the raw extents of blocks nx_b + lane
  // The sub-piece of blocks b0 + lane (lane < navail) from their raw extents:
  // this lane's extent, and (wave-uniform) the sub-piece's block count nb (0:
  // the first block alone spans >= 2 GiB), row base pb, descriptor window
  // [desc, desc + nrec) and rows NR.
  struct Plan {
    uint64_t sa, ea, bj;
    bool fits;
    uint64_t pb, desc;
    uint32_t nb, nrec, NR;
  };
  auto plan = [&](uint64_t b0, uint32_t navail, const ExtRaw& rq) -> Plan {
    Plan p;
    const bool vq = lane < navail;
    p.bj = vq ? b0 + lane : b0;
    uint64_t at;
    extent_from_raw(args, p.bj, rq, p.sa, p.ea, p.fits, at);
    // a record that does not fit is empty and bad; a well-formed batch
    // has such records only at its end, where the image ends
    if (!p.fits) p.sa = p.ea = base + args.limit;
    const uint64_t s_first = readlane64(p.sa, 0);
    p.pb = s_first & ~127ull;  // the sub-piece's row base (absolute, 128-aligned)
    // The sub-piece ends before the first block that is not in order (or
    // overlaps the one before; offsets that go back make an empty block
    // and then an earlier start) or that reaches 2 GiB past pb.
    const uint64_t pe = shfl_up64(p.ea, 1);
    bool cut = !vq || p.ea - p.pb >= (1ull << 31) - 4096u;  // (rows stay below the sentinel's)
    if (lane > 0) cut = cut || p.sa < pe;
    const uint64_t cm = __ballot(cut);
    p.nb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(cm ? (uint32_t)__builtin_ctzll(cm) : 64u));
    const uint32_t last = p.nb ? p.nb - 1u : 0u;
    const uint64_t e_last = readlane64(p.ea, last), s_last = readlane64(p.sa, last);
    p.desc = p.pb + ((uint32_t)(s_first - p.pb) & ~15u);  // chunks in [desc, roundup16(e_last)) are read
    p.nrec = (uint32_t)(((e_last + 15u) & ~15ull) - p.desc);
    p.NR = end_row((uint32_t)(s_last - p.pb), (uint32_t)(e_last - p.pb)) + 1u;
    // (wave-uniform: readfirstlane keeps the descriptor in SGPRs, with no
    // waterfall loop around the loads)
    p.desc = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p.desc) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p.desc >> 32)) << 32);
    p.nrec = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.nrec);
    p.pb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p.pb) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p.pb >> 32)) << 32);
    p.NR = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.NR);
    return p;
  };
  // Rows of a sub-piece: lane group g streams segment g of Q = ceil(NR / 8)
  // rows, one 16-B chunk per lane, two banks of kBank rows in flight.  Rows
  // past the segment are not read (the loop's last reloads, up to two banks
  // per group, would otherwise fetch the next group's rows again -- ~7% more
  // HBM reads on WAL records; an offset past the descriptor reads zeros
  // without a memory access).
  auto rows_of = [&](const Plan& p, uint32_t& Q, uint32_t& voff, __amdgpu_buffer_rsrc_t& rsrc) {
    Q = (p.NR + 7u) >> 3;
    voff = g * Q * (uint32_t)kRowBytes + 16u * li - (uint32_t)(p.desc - p.pb);  // (wraps: reads 0)
    rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(p.desc), (short)0, (int)p.nrec, 0x00020000);
  };
  auto ldr = [&](__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t Q, uint32_t r) -> u32x4 {
    const uint32_t off = r < Q ? voff + r * (uint32_t)kRowBytes : 0x80000000u;
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, kStreamAux));
  };
  u32x4 ba[kBank], bb[kBank];
  bool pre = false;  // the banks hold the next sub-piece's first rows already (issued before the tail)
  for (;;) {  // pieces (one, or this wave's range of every chunk)
    for (uint64_t b0 = b_lo; b0 < b_hi;) {
      // ---- the next sub-piece: up to 64 blocks in order (s_j >= e_{j-1}) ----
      LSBM_STAT(6, 1u);
      LSBM_TIC(0);
      const uint32_t navail = b_hi - b0 < kSubBlocks ? (uint32_t)(b_hi - b0) : kSubBlocks;
      uint32_t sr, er;  // relative to pb; er carries bit 31 for a record that does not fit
      uint64_t pb, desc;
      uint32_t nrec, NR, nb;
      uint32_t aux = 0;  // this lane's block's expected / stored CRC or type byte (loaded now, used at the end)
      {
        ExtRaw rq;
        if (nx_b == b0) {
          rq = nx;
        } else {
          rq = load_ext_raw(args, lane < navail ? b0 + lane : b0);
          if constexpr (kExt == kExtLogHeaders) {
            // Headers out of order already by their offsets (fewer than 16
            // ascending from b0): the units walk, without waiting for the
            // record lengths, a load that depends on these.
            const uint64_t prev = shfl_up64(rq.x, 1);
            const uint64_t down = __ballot(lane > 0u && lane < navail && rq.x <= prev);
            const uint32_t asc = down ? (uint32_t)__builtin_ctzll(down) : 64u;
            if (asc < kSubBlocks / 4u && asc < navail) {
              resume = b0;
              break;
            }
            log_length(args, rq);
          }
        }
        const Plan P = plan(b0, navail, rq);
        nb = P.nb;
        // The first block alone spans >= 2 GiB (nb == 0), or blocks out of
        // order (e.g. log headers passed by length, shuffled offsets): a
        // sub-piece of a few blocks would cost its setup and tail per block, so
        // the units walk takes the rest of the wave's range from b0 on.
        if (nb == 0u || (nb < kSubBlocks / 4u && nb < navail)) {
          resume = b0;
          break;
        }
        pb = P.pb;
        desc = P.desc;
        nrec = P.nrec;
        NR = P.NR;
        const uint64_t sa = P.sa, ea = P.ea, bj = P.bj;
        const bool fits = P.fits;
        sr = lane < nb ? (uint32_t)(sa - pb) : 0x7fffff00u;
        er = lane < nb ? (uint32_t)(ea - pb) | (fits ? 0u : 0x80000000u) : 0x7fffff00u;
        // the stored / written checksum: after the type byte, or in the log
        // header (6 bytes before the record's CRC bytes)
        const bool mine = lane < nb;
        uint64_t q = dummy;
        if constexpr (kMode == kModeVerify) q = mine ? reinterpret_cast<uint64_t>(args.expect + bj) : dummy;
        if constexpr (kMode == kModeSstCrc) q = mine ? reinterpret_cast<uint64_t>(args.types + bj) : dummy;
        if constexpr (kMode == kModeSstVerify) q = mine && fits ? ea : dummy;
        if constexpr (kMode == kModeLogVerify) q = mine && fits ? sa - 6u : dummy;
        if constexpr (kMode == kModeVerify) aux = *reinterpret_cast<gptr_u32>(q);
        if constexpr (kMode == kModeSstCrc) aux = *reinterpret_cast<gptr_u8>(q);
        if constexpr (kMode == kModeSstVerify || kMode == kModeLogVerify) aux = *reinterpret_cast<gptr_u32u>(q);
      }
      nx_b = b0 + nb;
      if (nx_b < b_hi) {  // (clamped as above)
        const uint64_t na = b_hi - nx_b < kSubBlocks ? b_hi - nx_b : kSubBlocks;
        nx = load_ext_raw(args, lane < na ? nx_b + lane : nx_b);
      } else {
        nx_b = ~0ull;
      }
      uint32_t Q, voff;  // rows per segment; this lane's first chunk in the descriptor
      __amdgpu_buffer_rsrc_t rsrc;
      rows_of(Plan{0, 0, 0, true, pb, desc, nb, nrec, NR}, Q, voff, rsrc);
      const uint32_t seg0 = g * Q;  // this group's first row (relative to pb)
      // ---- the segment's first two banks: issued now, so that their memory
      // latency runs under the rest of the setup (ballots, LDS picks) ----
      auto ld = [&](uint32_t r) -> u32x4 { return ldr(rsrc, voff, Q, r); };
      if (LSBM_STREAM_EARLY_BANKS && !pre) {
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) ba[k] = ld(k);
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) bb[k] = ld(kBank + k);
        pre = true;
      }
      // the first block of this group's segment: the number of blocks that
      // end before it; and the group where this lane's block ends (its lane 0:
      // the block's raw CRC is delivered from there)
      uint32_t cur = 0, fsrc = 0;
      {
        const uint32_t re = end_row(sr, er & 0x7fffffffu);
#pragma unroll
        for (uint32_t gg = 1; gg < 8; gg++) {
          const uint32_t f = (uint32_t)__builtin_popcountll(__ballot(lane < nb && re < gg * Q));
          cur = g == gg ? f : cur;
          fsrc += re >= gg * Q ? 32u : 0u;  // (bpermute address of lane 8 gg)
        }
      }
      uint32_t px = 0;  // this lane's block's raw CRC at the end of its last row

      // ---- the group's two pointers into the sub-piece's blocks ----
      // ep: the next block to end, sp: the next block to start (sp == ep + 1
      // while block ep is open).  E = the end of block ep, S = the start of
      // block sp with bit 31 set for a *short* block (one that starts and
      // ends in the same row; an empty block is short and its end is taken
      // as s + 1, so that it ends in its start row; its CRC does not use the
      // braids).  Lane j holds block j's values; lanes >= nb sentinels that
      // never start or end.  All group-uniform.
      constexpr uint32_t kShort = 0x80000000u;
      const uint32_t erm = er & 0x7fffffffu;
      const uint32_t ej = erm == sr ? sr + 1u : erm;
      const uint32_t sxl = sr | ((sr >> 7) == end_row(sr, erm) ? kShort : 0u);
      auto pick = [&](uint32_t v, uint32_t j) -> uint32_t {  // block j's value (every lane active;
        // j > 63: lane 63's sentinel)
        return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(j, 63u) << 2), (int)v);
      };
      uint32_t ep = cur, sp;
      {
        const uint32_t cs0 = pick(sr, ep);
        sp = ep < nb && (cs0 >> 7) < seg0 ? ep + 1u : ep;  // continued from the previous segment
      }
      uint32_t E = pick(ej, ep), S = pick(sxl, sp);
      uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
      // saved block ends: braids and block (relative to b0)
      uint32_t cnt = 0;
      uint32_t sx0[4] = {0, 0, 0, 0}, sx1[4] = {0, 0, 0, 0};
      uint32_t sb0 = 0, sb1 = 0;

      // Merge every group's oldest saved end (one merge_braids for all 8
      // groups) and hand each raw CRC to the lane of its block.  With two
      // slots the slots are a FIFO: a group that must save a third end frees
      // one slot in every group, so a merge takes the ends of most groups
      // rather than only of those that happened to end a block lately.
      auto merge_oldest = [&]() {  // every lane active
        LSBM_STAT(5, 1u);
        const uint32_t X = merge_braids(g_lds, sx0[0], sx0[1], sx0[2], sx0[3], lane_fin);
        // lane l takes the CRC of block l from the group where it ends
        const uint32_t bj = cnt != 0u ? sb0 : ~0u;
        const uint32_t xd = (uint32_t)__builtin_amdgcn_ds_bpermute((int)fsrc, (int)X);
        const uint32_t bd = (uint32_t)__builtin_amdgcn_ds_bpermute((int)fsrc, (int)bj);
        if (bd == lane) px = xd;
        if constexpr (kSlots == 2) {
          const bool two = cnt == 2u;
          sx0[0] = two ? sx1[0] : sx0[0];
          sx0[1] = two ? sx1[1] : sx0[1];
          sx0[2] = two ? sx1[2] : sx0[2];
          sx0[3] = two ? sx1[3] : sx0[3];
          sb0 = two ? sb1 : sb0;
        }
        cnt = cnt != 0u ? cnt - 1u : 0u;
      };
      auto flush = [&]() {  // room for one more end in every group
        LSBM_TIC(2);
        LSBM_STAT(4, 1u);
        if (__ballot(cnt != 0u) != 0ull) merge_oldest();
        LSBM_TOC(2);
      };
      // Save braids x of block b, which ends in this row, into the group's
      // next slot (ends: group-uniform; the caller made room).
      auto save = [&](bool ends, uint32_t b, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
        const bool s0 = ends && (kSlots == 1 || cnt == 0u), s1 = kSlots == 2 && ends && cnt == 1u;
        sx0[0] = s0 ? x0 : sx0[0];
        sx0[1] = s0 ? x1 : sx0[1];
        sx0[2] = s0 ? x2 : sx0[2];
        sx0[3] = s0 ? x3 : sx0[3];
        sb0 = s0 ? b : sb0;
        if constexpr (kSlots == 2) {
          sx1[0] = s1 ? x0 : sx1[0];
          sx1[1] = s1 ? x1 : sx1[1];
          sx1[2] = s1 ? x2 : sx1[2];
          sx1[3] = s1 ? x3 : sx1[3];
          sb1 = s1 ? b : sb1;
        }
        cnt += ends ? 1u : 0u;
      };
      auto km = [&](uint32_t lo, uint32_t hi) -> u32x4 {  // bytes [lo, hi) of a chunk
        return *reinterpret_cast<const u32x4*>(lds_c + kStreamHM + km_entry(lo, hi) * 16u);
      };
      auto clamp16 = [](uint32_t p, uint32_t rowa) -> uint32_t {  // p's offset in the chunk at rowa, in [0, 16]
        return (uint32_t)min(max((int32_t)p - (int32_t)rowa, 0), 16);
      };

      // Every row is the row step; a row where some group starts or ends a
      // block (nev, the group's next such row) is then fixed up.  A lean
      // fix-up handles at most one end (block ep, open) and one start (block
      // sp, not short) per group, as selects, with the LDS values it needs
      // read when the previous event was handled (hidden behind the rows in
      // between): mE = the bytes at or past E of this lane's chunk in row nev,
      // mS = those at or past S, iv = block sp's init register ~0 as injected
      // at its row start (A^-(S mod 128)(~0), util/crc32c.cc:289; lanes 1-7 of
      // a group read a zero word, the empty mask), En / Sn = the pointers'
      // next values.
      // erow: block ep's last row while it is open (~0 otherwise), srow: block
      // sp's first row, nev: the nearer of the two
      uint32_t nev, erow, srow;
      u32x4 mE, mS;
      uint32_t iv, En, Sn;
      // (the init register's LDS address: lane 0 of a group reads R0[S mod 128],
      // lanes 1-7 the zero word of the empty mask)
      const uint32_t iv_base = li == 0u ? kStreamR0 : kStreamHM + km_entry(16u, 16u) * 16u;
      const uint32_t iv_mask = li == 0u ? 127u : 0u;
      auto next_event = [&]() {
        erow = sp != ep ? (E - 1u) >> 7 : ~0u;
        srow = (S & ~kShort) >> 7;
        nev = min(erow, srow);
        const uint32_t rowa = nev * (uint32_t)kRowBytes + 16u * li;
        mE = *reinterpret_cast<const u32x4*>(lds_c + kStreamHM + clamp16(E, rowa) * 16u);
        mS = *reinterpret_cast<const u32x4*>(lds_c + kStreamHM + clamp16(S & ~kShort, rowa) * 16u);
        iv = *reinterpret_cast<const uint32_t*>(lds_c + iv_base + (S & iv_mask) * 4u);
        En = pick(ej, ep + 1u);
        Sn = pick(sxl, sp + 1u);
      };
      auto fix_lean = [&](u32x4 w, uint32_t rr) {  // after STEP_ROW: c = T(c) ^ w
        const bool e_in = erow == rr;
        const bool s_in = srow == rr;
        if (__ballot(e_in && cnt == kSlots) != 0ull) flush();
        LSBM_STAT(1, 1u);
        // block ep through E: T(c) ^ (w & bytes < E) = c ^ (w & mE)
        save(e_in, ep, __builtin_amdgcn_bitop3_b32(c0, w.x, mE.x, 0x78),
             __builtin_amdgcn_bitop3_b32(c1, w.y, mE.y, 0x78), __builtin_amdgcn_bitop3_b32(c2, w.z, mE.z, 0x78),
             __builtin_amdgcn_bitop3_b32(c3, w.w, mE.w, 0x78));
        // block sp from S: its bytes of the row and its init register
        c0 = s_in ? (w.x & mS.x) ^ iv : c0;
        c1 = s_in ? w.y & mS.y : c1;
        c2 = s_in ? w.z & mS.z : c2;
        c3 = s_in ? w.w & mS.w : c3;
        ep += e_in ? 1u : 0u;
        E = e_in ? En : E;
        sp += s_in ? 1u : 0u;
        S = s_in ? Sn : S;
        next_event();
      };

      // The general fix-up (a rolled loop runs it): any number of block ends
      // and starts, in order, flushing the slot as it fills up.
      auto fix_general = [&](u32x4 w, uint32_t rr) {  // after STEP_ROW
        LSBM_STAT(2, 1u);
        const uint32_t rowa = rr * (uint32_t)kRowBytes + 16u * li;
        // the open block: its braids through the row start and its bytes of
        // this row from lo on
        const bool open0 = sp != ep;
        uint32_t a0 = open0 ? c0 ^ w.x : 0u, a1 = open0 ? c1 ^ w.y : 0u;
        uint32_t a2 = open0 ? c2 ^ w.z : 0u, a3 = open0 ? c3 ^ w.w : 0u;
        uint32_t lo = 0;
        for (;;) {
          const bool open = sp != ep;
          const bool ev_end = open && ((E - 1u) >> 7) == rr;
          const bool ev_start = !open && ((S & ~kShort) >> 7) == rr;
          if (__ballot(ev_end || ev_start) == 0ull) break;
          LSBM_STAT(3, 1u);
          if (__ballot(ev_end && cnt == kSlots) != 0ull) flush();
          const u32x4 m = km(lo, max(clamp16(E, rowa), lo));
          save(ev_end, ep, a0 ^ (w.x & m.x), a1 ^ (w.y & m.y), a2 ^ (w.z & m.z), a3 ^ (w.w & m.w));
          const uint32_t inj = *reinterpret_cast<const uint32_t*>(lds_c + kStreamR0 + (S & 127u) * 4u);
          if (ev_start) {
            a0 = li == 0u ? inj : 0u;
            a1 = a2 = a3 = 0u;
            lo = clamp16(S & ~kShort, rowa);
          }
          ep += ev_end ? 1u : 0u;
          sp += ev_start ? 1u : 0u;
          const uint32_t nE = pick(ej, ep), nS = pick(sxl, sp);
          E = ev_end ? nE : E;
          S = ev_start ? nS : S;
        }
        if (sp != ep) {  // the block still open continues with its bytes [lo, 16) of the row
          const u32x4 m = km(lo, 16u);
          c0 = a0 ^ (w.x & m.x);
          c1 = a1 ^ (w.y & m.y);
          c2 = a2 ^ (w.z & m.z);
          c3 = a3 ^ (w.w & m.w);
        }
        next_event();
      };

      // ---- the segment: half-steps of kBank rows, two banks in flight ----
      if (!pre) {
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) ba[k] = ld(k);
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) bb[k] = ld(kBank + k);
      }
      pre = false;
      next_event();
      // Rows are fixed up lean until one where some group's next block to
      // start is short; from there the rest of the bank goes through the
      // general fix-up (one rolled copy of it).
      auto half = [&](u32x4 (&X)[kBank], uint32_t r) {
        const uint32_t rr0 = seg0 + r;
        uint32_t k0 = kBank;  // (wave-uniform)
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) {
          if (k0 == kBank && r + k < Q) {
            STEP_ROW(X[k]);
            LSBM_STAT(0, 1u);
            if (__ballot(nev == rr0 + k) != 0ull) {
              const bool gen = srow == rr0 + k && (S & kShort) != 0u;
              if (__builtin_expect(__ballot(gen) != 0ull, 0)) k0 = k;
              else fix_lean(X[k], rr0 + k);
            }
          }
        }
        if (k0 < kBank) {
          LSBM_TIC(3);
#pragma unroll 1
          for (uint32_t k = k0; k < kBank && r + k < Q; k++) {
            // (row k of the bank, k wave-uniform: a chain of selects, not an
            // indexed private array, which would go to scratch)
            const u32x4 w = k == 0 ? X[0] : k == 1 ? X[1 % kBank] : k == 2 ? X[2 % kBank]
                          : k == 3 ? X[3 % kBank] : k == 4 ? X[4 % kBank] : X[5 % kBank];
            static_assert(kBank <= 6, "rows of a bank: extend the select chain");
            if (k > k0) STEP_ROW(w);  // (row k0 has been stepped)
            fix_general(w, rr0 + k);
          }
          LSBM_TOC(3);
        }
      };
      LSBM_TOC(0);
      LSBM_TIC(1);
      // (the next sub-piece's record lengths: their header offsets arrive with
      // the first bank, and the loads queue behind the banks)
      if constexpr (kExt == kExtLogHeaders)
        if (nx_b != ~0ull) log_length(args, nx);
      // (the reloads are not skipped past the segment: a branch around them
      // makes the compiler's load counting merge pessimistically at the join,
      // and WAL records lost 3-4 points; loads past the segment fetch nothing)
      for (uint32_t r = 0; r < Q; r += 2 * kBank) {
        half(ba, r);
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) ba[k] = ld(r + 2 * kBank + k);
        if (r + kBank < Q) half(bb, r + kBank);
#pragma unroll
        for (uint32_t k = 0; k < kBank; k++) bb[k] = ld(r + 3 * kBank + k);
      }
      LSBM_TOC(1);
      LSBM_TIC(5);
      // ---- blocks that cross segments ----
      // T: the braids of the block still open at the segment end, shifted to
      // that block's last row; summed per block over consecutive groups, and
      // added to the block's CRC in the lane that finishes it.  (The column
      // load first: the last flush hides its latency.)
      const bool tvalid = sp != ep && ep < nb;
      const uint32_t kt = tvalid ? ((E - 1u) >> 7) - (seg0 + Q - 1u) : 0u;  // rows to its last row
      const u32x4 scols = *reinterpret_cast<gptr_u32x4>(
          reinterpret_cast<uint64_t>(&dc->shift_cols[kt & (kShiftCols - 1u)][4 * li]));
      // ---- the next sub-piece's first rows, before this one's tail ----
      // (its extents, and log record lengths, have arrived during the row
      // loop; the tail's latency -- merges, the finishing chain -- then
      // overlaps its first loads instead of leaving the wave with nothing in
      // flight.  Issued after the tail's column load, which the tail waits for:
      // s_waitcnt counts vector loads in issue order)
      if (LSBM_STREAM_PREISSUE && nx_b != ~0ull) {
        const uint32_t na = b_hi - nx_b < kSubBlocks ? (uint32_t)(b_hi - nx_b) : kSubBlocks;
        const Plan P = plan(nx_b, na, nx);
        if (P.nb != 0u && !(P.nb < kSubBlocks / 4u && P.nb < na)) {
          uint32_t Q2, voff2;
          __amdgpu_buffer_rsrc_t rsrc2;
          rows_of(P, Q2, voff2, rsrc2);
#pragma unroll
          for (uint32_t k = 0; k < kBank; k++) ba[k] = ldr(rsrc2, voff2, Q2, k);
#pragma unroll
          for (uint32_t k = 0; k < kBank; k++) bb[k] = ldr(rsrc2, voff2, Q2, kBank + k);
          pre = true;
        }
      }
      uint32_t xt;
      if constexpr (kSlots == 2 && LSBM_STREAM_MERGE2)  // (the paired merge takes the last one)
        if (__ballot(cnt == 2u) != 0ull) merge_oldest();
      if constexpr (LSBM_STREAM_MERGE2) {
        // the last saved ends and the open block's braids, merged together
        uint32_t X;
        merge_braids2(g_lds, sx0[0], sx0[1], sx0[2], sx0[3], c0, c1, c2, c3, lane_fin, X, xt);
        const uint32_t bj = cnt != 0u ? sb0 : ~0u;
        const uint32_t xd = (uint32_t)__builtin_amdgcn_ds_bpermute((int)fsrc, (int)X);
        const uint32_t bd = (uint32_t)__builtin_amdgcn_ds_bpermute((int)fsrc, (int)bj);
        if (bd == lane) px = xd;
        cnt = 0;
      } else {
        while (__ballot(cnt != 0u) != 0ull) merge_oldest();
        xt = merge_braids(g_lds, c0, c1, c2, c3, lane_fin);
      }
      xt = cols_apply(scols, xt, li);
      if (tvalid && kt >= kShiftCols) xt = shift_rows(g_lds, dc, xt, kt & ~(kShiftCols - 1u));
      uint32_t v = tvalid ? xt : 0u;
      const uint32_t key = tvalid ? ep : ~0u;
#pragma unroll
      for (uint32_t d = 8; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, d);
        const uint32_t tk = (uint32_t)__shfl_up((int)key, d);
        if (lane >= d && tk == key) v ^= t;
      }
      {  // the pieces summed up to the group before the one where block `lane` ends
        const uint32_t pv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fsrc - 32u), (int)v);
        const uint32_t pk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fsrc - 32u), (int)key);
        if (fsrc != 0u && pk == lane) px ^= pv;
      }
      LSBM_TIC(6);
      // ---- finish: lane l, block b0 + l ----
      {
        const bool mine = lane < nb;
        const uint32_t be = er & 0x7fffffffu;
        const bool bad = (er >> 31) != 0u;
        const bool empty = sr == be;
        const uint32_t z = (0u - be) & 127u;  // bytes of the last row after e (pb is 128-aligned)
        // A^-z, or A^(1-z) when the type byte follows (WriteRawBlock's Extend),
        // as A^-128 A^m, m = 128 - z (+1): the LDS power tables, bit by bit
        const uint32_t m = (kMode == kModeSstCrc ? 129u : 128u) - z;
        uint32_t l = nib_lds_at(g_lds, kNibNeg128, px);
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) {
          const uint32_t t = nib_lds_at(g_lds, kNibPow2 + i * 512u, l);
          l = ((m >> i) & 1u) ? t : l;
        }
        // an empty block leaves the init register ~0 (advanced by the type byte's slot)
        if (empty) l = kMode == kModeSstCrc ? advance_byte(0xffffffffu) : 0xffffffffu;
        const uint32_t crc = l ^ 0xffffffffu;
        const uint64_t bi = b0 + lane;
        if constexpr (kMode == kModeOut) {
          if (mine) args.out[bi] = (args.flags & 1u) ? mask_crc(crc) : crc;
        } else if constexpr (kMode == kModeVerify) {
          const bool good = ((args.flags & 1u) ? mask_crc(crc) : crc) == aux;
          nbad += (uint32_t)__builtin_popcountll(__ballot(mine && !good));
          if (mine) args.ok[bi] = good ? 1u : 0u;
        } else if constexpr (kMode == kModeSstCrc) {  // table/table_builder.cc:245-249
          nbad += (uint32_t)__builtin_popcountll(__ballot(mine && bad));
          if (mine) args.out[bi] = bad ? 0u : mask_crc((l ^ advance_byte(aux & 0xffu)) ^ 0xffffffffu);
        } else if constexpr (kMode == kModeLogSeal) {  // common/log_writer.cc:85-88
          nbad += (uint32_t)__builtin_popcountll(__ballot(mine && bad));
          const uint32_t val = mask_crc(crc);
          if (mine && !bad && args.file && !(args.flags & kFlagDeferHeaders)) {  // header[0..4): one unaligned dword store
            typedef __attribute__((address_space(1), aligned(1))) uint32_t* gu32u;
            *reinterpret_cast<gu32u>(pb + sr - 6u) = val;
          }
          if (mine && args.out) args.out[bi] = bad ? 0u : val;
        } else {  // kModeSstVerify (table/format.cc:95-103), kModeLogVerify (log_reader.cc:228-242)
          const bool good = !bad && unmask_crc(aux) == crc;
          nbad += (uint32_t)__builtin_popcountll(__ballot(mine && !good));
          if (mine) args.ok[bi] = good ? 1u : 0u;
        }
      }
      LSBM_TOC(6);
      LSBM_TOC(5);
      b0 += nb;
    }
    if (!chunked || resume != ~0ull) break;
    pi = claim ? next_piece<kStreamWavesPerWg>(claim, pi, nwaves) : pi + (uint32_t)nwaves;
    if (pi >= p_end) break;
    piece_range(args, pi, p_end, b_lo, b_hi);
  }
#ifdef LSBM_STREAM_STATS
  if (lane == 0u)
    for (int i = 0; i < 8; i++) {
      atomicAdd(&g_stream_stats[i], (unsigned long long)st[i]);
      atomicAdd(&g_stream_stats[8 + i], (unsigned long long)tm[i]);
    }
#endif
  if (resume != ~0ull) {
    // The units walk from block `resume` on: the rest of this range, then (a
    // chunked sweep) this wave's range of every later chunk.  Its bad blocks
    // are counted by the walk; this wave's nbad holds the streamed ones.
    if constexpr (kCanChunk<kMode, kExt>) {
      if (claim)
        units_walk<kFallbackRows, kMode, kExt, true, kStreamWavesPerWg>(args, wave, nwaves, resume, b_hi, chunked, pi,
                                                                        p_end, false, resume, claim);
      else
        units_walk<kFallbackRows, kMode, kExt>(args, wave, nwaves, resume, b_hi, chunked, pi, p_end, false, resume);
    } else {
      units_walk<kFallbackRows, kMode, kExt>(args, wave, nwaves, resume, b_hi, chunked, pi, p_end, false, resume);
    }
  }
  if constexpr (kMode == kModeLogSeal) {
    // Deferred headers: this wave's masked CRCs went densely to out[] with
    // its reads; the scattered header stores follow its last row, so they do
    // not sit in the in-order load counter between the streamed rows (the
    // SSTable seal's trailer epilogue, crc32c_kernels.hip).  (Not chunked:
    // [b_lo, b_hi) is the wave's whole range.)
    if ((args.flags & kFlagDeferHeaders) && args.file) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's out[] stores performed
      typedef __attribute__((address_space(1), aligned(1))) uint32_t* gu32u;
      // (the units walk wrote the headers of [resume, b_hi) in place)
      const uint64_t d_hi = resume < b_hi ? resume : b_hi;
      for (uint64_t i = b_lo + lane; i < d_hi; i += 64u) {
        ExtRaw r = load_ext_raw(args, i);
        uint64_t at = base + r.x;
        bool fits = true;
        if (nbad != 0u) {  // (only a wave with a record that does not fit reads the lengths again)
          log_length(args, r);
          uint64_t s, e;
          extent_from_raw(args, i, r, s, e, fits, at);
        }
        if (fits) {
          const uint32_t v = __hip_atomic_load(args.out + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *reinterpret_cast<gu32u>(reinterpret_cast<uint64_t>(args.file) + (at - base)) = v;  // header[0..4)
        }
      }
    }
  }
  if (lane == 0u && nbad && args.nbad) atomicAdd(args.nbad, nbad);
  DIAG_STAMP_W(2, wave);
  DIAG_XCC_W(wave);
}

// Which batches go this way: no per-block init (crc32c::Value semantics;
// init injection is a table lookup), and one of the modes below.
bool stream_eligible(const RaggedArgs& a) {
  if (a.init || a.n >= 0xffffff00ull) return false;  // (block indices are 32-bit in the kernel)
  switch (a.mode) {
    case kModeOut: return a.extents == kExtOffsets || a.extents == kExtHandles;
    case kModeVerify: return a.extents == kExtOffsets;
    case kModeSstCrc: return a.extents == kExtHandles && !a.file;  // (the fused seal: units kernel)
    case kModeSstVerify: return a.extents == kExtHandles;
    case kModeLogSeal:
    case kModeLogVerify: return a.extents == kExtLogHeaders;
    default: return false;
  }
}

hipError_t launch_stream(const RaggedArgs& a, int grid, hipStream_t stream) {
#define LSBM_LAUNCH_STREAM(R, M, X) \
  hipLaunchKernelGGL((crc32c_stream_kernel<R, M, X>), dim3(grid), dim3(kStreamThreads), 0, stream, a)
  switch (a.mode) {
    case kModeOut:
      if (a.extents == kExtOffsets) LSBM_LAUNCH_STREAM(32, kModeOut, kExtOffsets);
      else LSBM_LAUNCH_STREAM(32, kModeOut, kExtHandles);
      break;
    case kModeVerify: LSBM_LAUNCH_STREAM(32, kModeVerify, kExtOffsets); break;
    case kModeSstCrc: LSBM_LAUNCH_STREAM(32, kModeSstCrc, kExtHandles); break;
    case kModeSstVerify: LSBM_LAUNCH_STREAM(32, kModeSstVerify, kExtHandles); break;
    case kModeLogSeal: LSBM_LAUNCH_STREAM(16, kModeLogSeal, kExtLogHeaders); break;
    case kModeLogVerify: LSBM_LAUNCH_STREAM(16, kModeLogVerify, kExtLogHeaders); break;
    default: return hipErrorInvalidValue;
  }
#undef LSBM_LAUNCH_STREAM
  return hipGetLastError();
}

}  // namespace lsbm

#ifdef LSBM_DIAG_STAMPS
// diagnostic builds only: the stream kernel's per-wave timeline (crc32c_units.h)
extern "C" __attribute__((visibility("default"))) int lsbm_diag_stamps_stream(uint64_t* host, int n) {
  (void)n;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lsbm::g_stamps), sizeof(uint64_t) * 4 * 65536) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LSBM_STREAM_STATS
// diagnostic builds only: read and clear the counters
extern "C" __attribute__((visibility("default"))) int lsbm_stream_stats(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lsbm::g_stream_stats), sizeof(unsigned long long) * 16) != hipSuccess)
    return -1;
  unsigned long long z[16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(lsbm::g_stream_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
