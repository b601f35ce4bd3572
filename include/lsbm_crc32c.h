/*
 * lsbm_crc32c.h -- C ABI of the MI355X (gfx950) batched CRC-32C engine for
 * lsbm's block checksums.  Implemented by lsbm_amd/liblsbm_crc32c.so.
 *
 * Every entry point is extern "C", takes plain pointers and sizes, never throws
 * and never aborts.  Status codes are the LSBM_* values below (0 = ok).
 * Device (`_dev`) entry points take device pointers and an explicit HIP stream
 * (`void* stream` is a hipStream_t; NULL = the legacy default stream); they
 * only enqueue work, never synchronise, and may be captured into a hipGraph
 * once the device has been initialised with lsbm_crc32c_init().
 * They are thread-safe: per-device tables are built once (on first use) and
 * are read-only until lsbm_crc32c_shutdown(); callers serialise through their
 * own streams.
 *
 * Reference interfaces replaced (lsbm = tengdj/lsbm, a LevelDB 1.15 fork):
 *   util/crc32c.h:17-40      crc32c::Extend / Value / Mask / Unmask
 *                            -> lsbm_crc32c_extend/_value/_mask/_unmask (scalar)
 *                               and include/util/crc32c.h (same C++ API)
 *   util/crc32c.cc:286-329   the per-block Extend loop, batched
 *                            -> lsbm_crc32c_fixed_dev / lsbm_crc32c_batch_dev
 *   table/table_builder.cc:237-255  TableBuilder::WriteRawBlock trailer seal
 *                            -> lsbm_sst_seal_dev
 *   table/format.cc:95-103   ReadBlock's verify_checksums compare
 *                            -> lsbm_sst_verify_dev
 *   table/format.h:84        kBlockTrailerSize = 5 -> LSBM_BLOCK_TRAILER_SIZE
 *   common/log_writer.cc:75-100  log::Writer::EmitPhysicalRecord header CRC
 *                            -> lsbm_log_seal_dev
 *   common/log_reader.cc:228-242 log::Reader::ReadPhysicalRecord checksum
 *                            -> lsbm_log_verify_dev
 */
#ifndef LSBM_CRC32C_H_
#define LSBM_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define LSBM_OK 0
#define LSBM_ERR_INVALID (-1)     /* bad argument (null pointer, size, flags) */
#define LSBM_ERR_NO_DEVICE (-2)   /* no HIP device / bad device ordinal */
#define LSBM_ERR_HIP (-3)         /* a HIP runtime call failed */
#define LSBM_ERR_NOMEM (-4)       /* device or pinned allocation failed */
#define LSBM_ERR_CORRUPTION (-5)  /* verify found >= 1 mismatching block */

/* ---- flags ---- */
#define LSBM_CRC32C_MASKED 0x1u /* out = Mask(crc) (util/crc32c.h:31-34) */

#define LSBM_CRC32C_MASK_DELTA 0xa282ead8u /* util/crc32c.h:24 kMaskDelta */
#define LSBM_BLOCK_TRAILER_SIZE 5          /* table/format.h:84 */

/* ---- scalar API: identical results to util/crc32c.{h,cc}; host CPU ---- */
uint32_t lsbm_crc32c_extend(uint32_t init_crc, const char* data, size_t n);
uint32_t lsbm_crc32c_value(const char* data, size_t n);
uint32_t lsbm_crc32c_mask(uint32_t crc);
uint32_t lsbm_crc32c_unmask(uint32_t masked_crc);

/* ---- engine ---- */
/* Builds the per-device tables (idempotent, thread-safe).  Optional: every
 * _dev call initialises lazily, but graph capture needs it done beforehand. */
int lsbm_crc32c_init(int device);
/* Frees everything the library holds on every device: the tables, the
 * host-staged batch slots and the C++ layers' staging (pinned and device
 * buffers, streams).  Call it with no library work in flight or pending
 * (it synchronises the devices it touches); the next call re-initialises. */
int lsbm_crc32c_shutdown(void);
/* Library version string and the last HIP error text seen on this thread. */
const char* lsbm_crc32c_version(void);
const char* lsbm_crc32c_last_error(void);

/* Fixed-stride batch: block i = d_base[i*stride, i*stride + len).
 * out[i] = Extend(init ? init[i] : 0, block i, len), Mask()ed if flags has
 * LSBM_CRC32C_MASKED.  d_init may be NULL (crc32c::Value).  Any stride/len;
 * 16-B aligned base, stride % 16 == 0 and len % 128 == 0 take the fast path. */
int lsbm_crc32c_fixed_dev(const void* d_base, uint64_t stride, uint64_t len, uint64_t n_blocks,
                          const uint32_t* d_init, uint32_t* d_out, uint32_t flags, void* stream);

/* Ragged batch: block i = d_base[offsets[i], offsets[i+1]) (d_offsets has
 * n_blocks+1 entries, non-decreasing not required; any alignment).
 * Big batches (this, extents and verify; from 8 x 128 blocks per wave of the
 * device, 4.2M blocks on an MI355X) are swept chunk by chunk: a first small
 * launch on the stream writes the chunks' ranges into ~n_blocks / 32 bytes
 * of stream-ordered scratch (hipMallocAsync from the device's default pool,
 * freed on the stream after the CRC launch).  Without it, or while the
 * stream is being captured, one launch as for smaller batches. */
int lsbm_crc32c_batch_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n_blocks,
                          const uint32_t* d_init, uint32_t* d_out, uint32_t flags, void* stream);

/* Extent-list batch: block i = d_base[ext[2i], ext[2i] + ext[2i+1]) ({offset,
 * length} pairs, any order, may overlap).  For records that are not
 * contiguous, e.g. WAL payloads between their 7-byte headers: with
 * d_init[i] = type_crc_[t] and LSBM_CRC32C_MASKED this is exactly
 * log::Writer::EmitPhysicalRecord's header CRC (common/log_writer.cc:86-87). */
int lsbm_crc32c_extents_dev(const void* d_base, const uint64_t* d_extents, uint64_t n_blocks,
                            const uint32_t* d_init, uint32_t* d_out, uint32_t flags, void* stream);

/* Ragged verify: d_ok[i] = (crc of block i == d_expect[i]) where d_expect holds
 * masked values if flags has LSBM_CRC32C_MASKED.  If d_nbad != NULL the
 * number of mismatches is ADDED to *d_nbad (caller zeroes it). */
int lsbm_crc32c_verify_dev(const void* d_base, const uint64_t* d_offsets, uint64_t n_blocks,
                           const uint32_t* d_init, const uint32_t* d_expect, uint8_t* d_ok,
                           uint32_t* d_nbad, uint32_t flags, void* stream);

/* ---- SSTable block trailers over a device-resident file image ----
 * d_file is file_bytes long; d_handles holds n_blocks BlockHandles as
 * {offset, size} uint64 pairs (table/format.h:22-50).  The block occupies
 * file[offset, offset+size) and its 5-byte trailer
 * [type u8][Mask(crc32c(block || type)) LE32] follows it.  A handle whose
 * size + 5 bytes do not fit inside file_bytes is ReadBlock's "truncated block
 * read" (table/format.cc:88-91): no byte of it is read or written, it is
 * counted into *d_nbad (when non-NULL) and, for verify, d_ok[i] = 0.  Callers
 * that need to tell it from a checksum mismatch compare the handle with
 * file_bytes (include/lsbm/table_checksum.h does). */
/* WriteRawBlock (table/table_builder.cc:237-255): write each trailer, with
 * type = d_types[i] (CompressionType, include/leveldb/options.h:24-29).
 * One launch on the stream: the CRCs into 4 * n_blocks bytes of
 * stream-ordered scratch (hipMallocAsync from the device's default pool,
 * which lsbm_crc32c_init() sets to keep freed memory), after which each wave
 * merges its own blocks' trailers (written in place as they are computed if
 * that scratch cannot be had, e.g. under graph capture). */
int lsbm_sst_seal_dev(uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles,
                      const uint8_t* d_types, uint64_t n_blocks, uint32_t* d_nbad, void* stream);
/* The same trailers without touching the image: d_masked[i] =
 * Mask(Extend(Value(block i), &d_types[i], 1)), the 4 bytes WriteRawBlock
 * stores after the type byte (0 for a handle past the image, counted into
 * *d_nbad).  The output is dense, 4 B per block: scattered 5-byte writes into
 * the image cost the memory system more than the whole CRC read (DESIGN.md
 * section 3), so a host that writes the file itself wants this one. */
int lsbm_sst_trailer_crcs_dev(const uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles,
                              const uint8_t* d_types, uint64_t n_blocks, uint32_t* d_masked,
                              uint32_t* d_nbad, void* stream);
/* ReadBlock verify (table/format.cc:95-103): d_ok[i] = 1 iff the block fits and
 * Unmask(DecodeFixed32(trailer+1)) == Value(block || type); failures are
 * added to *d_nbad when non-NULL. */
int lsbm_sst_verify_dev(const uint8_t* d_file, uint64_t file_bytes, const uint64_t* d_handles,
                        uint64_t n_blocks, uint8_t* d_ok, uint32_t* d_nbad, void* stream);

/* ---- WAL / MANIFEST log records over a device-resident log image ----
 * common/log_format.h: 32 KiB log blocks of physical records, each a 7-byte
 * header [masked crc LE32][length LE16][type u8] followed by `length` payload
 * bytes.  d_headers[i] is the byte offset of record i's header in d_log
 * (log_bytes long); the CRC covers [type || payload] = header[6, 7 + length).
 * A record whose header or payload does not fit inside log_bytes is counted
 * into *d_nbad (when non-NULL) and never read past the image. */
/* log::Writer::EmitPhysicalRecord (common/log_writer.cc:75-100): with length
 * and type already in place, writes header[0, 4) =
 * EncodeFixed32(Mask(Extend(type_crc_[type], payload, length))), which equals
 * Mask(Value(header + 6, 1 + length)); d_masked (nullable) receives the same
 * masked values.  Records that do not fit are left untouched (d_masked 0). */
int lsbm_log_seal_dev(uint8_t* d_log, uint64_t log_bytes, const uint64_t* d_headers,
                      uint64_t n_records, uint32_t* d_masked, uint32_t* d_nbad, void* stream);
/* The same masked CRCs into d_masked (required) without writing the image:
 * for a host that frames the log itself (include/lsbm/log_checksum.h). */
int lsbm_log_crcs_dev(const uint8_t* d_log, uint64_t log_bytes, const uint64_t* d_headers,
                      uint64_t n_records, uint32_t* d_masked, uint32_t* d_nbad, void* stream);
/* log::Reader::ReadPhysicalRecord's checksum (common/log_reader.cc:228-242):
 * d_ok[i] = 1 iff the record fits and
 * Unmask(DecodeFixed32(header)) == Value(header + 6, 1 + length). */
int lsbm_log_verify_dev(const uint8_t* d_log, uint64_t log_bytes, const uint64_t* d_headers,
                        uint64_t n_records, uint8_t* d_ok, uint32_t* d_nbad, void* stream);

/* ---- host-staged batch (blocks start and end in host memory) ----
 * Same contract as lsbm_crc32c_batch_dev but every pointer is a host pointer
 * (pageable or pinned).  Bytes are streamed through pinned staging buffers
 * with hipMemcpyAsync overlapped with the kernel; blocks on `device`.
 * Synchronous: returns when h_out is filled. */
int lsbm_crc32c_batch_host(int device, const void* h_base, const uint64_t* h_offsets,
                           uint64_t n_blocks, const uint32_t* h_init, uint32_t* h_out,
                           uint32_t flags);

/* The same over several devices: the blocks are cut into contiguous shards
 * of about equal bytes, one per devices[k], each checksummed by its own host
 * thread through its own device's staging and streams.  No collective and no
 * device-to-device traffic: blocks are independent. */
int lsbm_crc32c_batch_host_multi(const int* devices, int n_devices, const void* h_base,
                                 const uint64_t* h_offsets, uint64_t n_blocks,
                                 const uint32_t* h_init, uint32_t* h_out, uint32_t flags);

/* ---- device helpers ----
 * d_dst[d_dst_off[i], +d_len[i]) = d_src[d_src_off[i], +d_len[i]) for i < n
 * (segments must not overlap each other's destinations): compacts
 * variable-length results before a D2H copy. */
int lsbm_gather_dev(const void* d_src, const uint64_t* d_src_off, const uint64_t* d_len, uint64_t n,
                    void* d_dst, const uint64_t* d_dst_off, void* stream);

/* ---- benchmark / diagnostic helpers (not on the checksum path) ---- */
/* d_buf[k] = byte k of the splitmix64 stream `seed`. */
int lsbm_fill_splitmix64_dev(void* d_buf, uint64_t nbytes, uint64_t seed, void* stream);
/* Reads nbytes (16-B aligned, multiple of 16) once, with the CRC kernels' own
 * access pattern (8 x 4 KiB blocks per wave as 128-B rows, 16-B non-temporal
 * loads), into d_sink[0..1023]: the measured read ceiling for that pattern. */
int lsbm_stream_read_dev(const void* d_buf, uint64_t nbytes, uint32_t* d_sink, void* stream);

/* ---- testing ---- */
/* Fault injection for the host layers' error-path tests: the next pipeline of
 * SealTables / VerifyTables / the log layer returns IOError("injected fault")
 * after enqueueing `chunks` chunks, as a failed copy or launch would (-1:
 * disarm).  Not for production use. */
int lsbm_test_fail_host_pipeline(int chunks);
/* Ragged-batch kernel policy (what LSBM_RAGGED_KERNEL sets at start-up): 0 the
 * default (the stream kernel for offsets[] batches and for log record headers,
 * the units kernel for fixed-stride, {offset, length} extents and SSTable
 * handles), 1 the units kernel for every batch, 2 the stream kernel for every
 * batch it takes.  Results are identical; for tests and A/B runs. */
int lsbm_test_ragged_kernel(int which);

/* Testing / A/B: the fixed-stride kernel's cross-XCC work queue on (1) or off
 * (0, the static interleave); -1 restores the default (LSBM_FIXED_QUEUE,
 * off). */
int lsbm_test_fixed_queue(int on);
/* Testing / A/B: SSTable trailer batches (verify, dense trailer CRCs) as
 * equal-count pieces claimed by a workgroup's waves (1) or one range per wave
 * (0); -1 restores the default (LSBM_SST_PIECES, one range per wave). */
int lsbm_test_sst_pieces(int on);

/* ---- host runtime (the C++ layers' sessions and worker pool) ---- */
/* Worker threads of the host pool: usable cores - 1, where usable cores = the
 * affinity mask capped by the cgroup CPU quota (LSBM_HOST_THREADS overrides);
 * starts the pool. */
int lsbm_host_threads(void);

/* Long-lived page-locking of a host buffer that is reused from call to call
 * (an embedder's table-image pool, integration/image_pool.h), inside the
 * library's own page-lock bookkeeping: the buffer's pages are reserved, so no
 * call page-locks over them and no other range on one of them is DMA-ed in
 * place (its owner may unregister at any time), while a range inside the
 * registered bytes is.  Refused (-1, nothing done) when a page of the range
 * belongs to a live call's lock or to another registration, when either end
 * is registered already, or past LSBM_PINNED_MB of such registrations.  No
 * reference counterpart: lsbm pins nothing (host-side plumbing). */
int lsbm_host_register(const void* p, uint64_t n);
int lsbm_host_unregister(const void* p); /* p as registered; 0 or -1 */
unsigned long long lsbm_host_registered_bytes(void);
/* NUMA node of HIP device `device` (from its PCI bus id and
 * /sys/bus/pci/devices/<id>/numa_node), -1 if unknown. */
int lsbm_device_numa_node(int device);
/* Testing: the same lookup under another sysfs root; cpulist parsing ("0-3,8"
 * -> up to cap CPUs, returns the count or -1 if malformed); the cgroup quota
 * under another cgroup root (whole CPUs, 0 if none); and the pool under load:
 * `callers` threads each run `jobs` parallel jobs of `pieces` pieces that each
 * sleep `piece_us`; returns the most jobs that had pieces running at once and
 * stores the wall seconds in *seconds. */
int lsbm_test_pci_numa_node(const char* sysfs_root, const char* bus_id);
int lsbm_test_parse_cpulist(const char* list, int* cpus, int cap);
int lsbm_test_cgroup_quota(const char* cgroup_root);
int lsbm_test_pool_overlap(int callers, int jobs, int pieces, int piece_us, double* seconds);
/* Testing: the quota of the process's own cgroup as usable_cores() finds it:
 * `proc_cgroup` is the text of /proc/self/cgroup, resolved under the cgroup
 * mount `cgroup_root` (the smallest quota over the cgroup and its ancestors;
 * the mount root's when none). */
int lsbm_test_cgroup_quota_of(const char* cgroup_root, const char* proc_cgroup);
/* Testing: one job of `pieces` pieces that each sleep `piece_us`, with at
 * most `max_helpers` pool workers joining the caller (-1: any number);
 * returns how many distinct threads ran its pieces. */
int lsbm_test_pool_helpers(int pieces, int piece_us, int max_helpers);
/* Testing: page ranges currently page-locked by the C++ layers' per-call
 * locks (0 whenever no call is running), and how many ranges they have
 * page-locked since start-up (which calls DMA-ed an image in place). */
int lsbm_test_locked_ranges(void);
long lsbm_test_locks_taken(void);
/* Testing: the C++ layers' sessions of `device`, and the page-locked staging
 * bytes they hold (kept near LSBM_PINNED_MB per device by freeing idle
 * sessions' buffers when a lease is released). */
int lsbm_test_session_count(int device);
unsigned long long lsbm_test_pinned_bytes(int device);
/* Testing: `callers` threads each run `jobs` parallel jobs of 1..max_pieces
 * pieces (some with nested jobs); returns how many pieces did not run exactly
 * once (0 = correct), -1 for bad arguments. */
int lsbm_test_pool_stress(int callers, int jobs, int max_pieces);
/* Testing: 1 if the C++ layers would DMA [p, p + n) in place (page-locked by
 * hipHostMalloc or one hipHostRegister covering the whole range, and no page
 * of it held by another call's per-call lock), else 0. */
int lsbm_test_host_pinned(const void* p, size_t n);
/* Testing: page-locked table jobs up to `mb` MiB take the small-job path
 * (each table one whole-image DMA and one kernel on a stage's stream, or with
 * LSBM_SMALL_LOCKED=zc read by the kernel in place) instead of the chunk
 * pipeline (LSBM_ZERO_COPY_MAX_MB sets it at start-up; 0 = never); returns -1
 * for mb < 0. */
int lsbm_test_zero_copy_max_mb(int mb);
/* Testing / measurement: the pageable layers' staging copy of n bytes (src ->
 * dst, non-temporal stores), over the worker pool when `parallel` is nonzero,
 * else on the calling thread.  Returns 0. */
int lsbm_test_host_copy(void* dst, const void* src, size_t n, int parallel);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* LSBM_CRC32C_H_ */
