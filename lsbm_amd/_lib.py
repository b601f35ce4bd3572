"""Loader for the product library lsbm_amd/liblsbm_crc32c.so (ctypes, C ABI).

Fails loudly when the library is missing: there is no CPU fallback for any
batch entry point (include/lsbm_crc32c.h).  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C lsbm_amd/csrc``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblsbm_crc32c.so")
# diagnostic builds (tools/ablate_units.sh) are loaded through LSBM_LIB_PATH
LIB_PATH = os.environ.get("LSBM_LIB_PATH") or LIB_PATH

# status codes (include/lsbm_crc32c.h)
LSBM_OK = 0
LSBM_ERR_INVALID = -1
LSBM_ERR_NO_DEVICE = -2
LSBM_ERR_HIP = -3
LSBM_ERR_NOMEM = -4
LSBM_ERR_CORRUPTION = -5
LSBM_CRC32C_MASKED = 0x1
LSBM_CRC32C_MASK_DELTA = 0xA282EAD8
LSBM_BLOCK_TRAILER_SIZE = 5

# every symbol include/lsbm_crc32c.h and include/lsbm_bloom.h declare: name -> (restype, argtypes)
_u32, _u64, _int, _vp, _sz = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_size_t)
SIGNATURES = {
    "lsbm_crc32c_extend": (_u32, [_u32, _vp, _sz]),
    "lsbm_crc32c_value": (_u32, [_vp, _sz]),
    "lsbm_crc32c_mask": (_u32, [_u32]),
    "lsbm_crc32c_unmask": (_u32, [_u32]),
    "lsbm_crc32c_init": (_int, [_int]),
    "lsbm_crc32c_shutdown": (_int, []),
    "lsbm_crc32c_version": (ctypes.c_char_p, []),
    "lsbm_crc32c_last_error": (ctypes.c_char_p, []),
    "lsbm_crc32c_fixed_dev": (_int, [_vp, _u64, _u64, _u64, _vp, _vp, _u32, _vp]),
    "lsbm_crc32c_batch_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _u32, _vp]),
    "lsbm_crc32c_extents_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _u32, _vp]),
    "lsbm_crc32c_verify_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _vp, _u32, _vp]),
    "lsbm_sst_seal_dev": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    "lsbm_sst_verify_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_sst_trailer_crcs_dev": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_log_seal_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_log_verify_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_log_crcs_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_crc32c_batch_host": (_int, [_int, _vp, _vp, _u64, _vp, _vp, _u32]),
    "lsbm_crc32c_batch_host_multi": (_int, [_vp, _int, _vp, _vp, _u64, _vp, _vp, _u32]),
    "lsbm_gather_dev": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_fill_splitmix64_dev": (_int, [_vp, _u64, _u64, _vp]),
    "lsbm_stream_read_dev": (_int, [_vp, _u64, _vp, _vp]),
    "lsbm_test_fail_host_pipeline": (_int, [_int]),
    "lsbm_test_ragged_kernel": (_int, [_int]),
    "lsbm_test_fixed_queue": (_int, [_int]),
    "lsbm_test_sst_pieces": (_int, [_int]),
    "lsbm_host_threads": (_int, []),
    "lsbm_host_register": (_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "lsbm_host_unregister": (_int, [ctypes.c_void_p]),
    "lsbm_host_registered_bytes": (ctypes.c_ulonglong, []),
    "lsbm_device_numa_node": (_int, [_int]),
    "lsbm_test_pci_numa_node": (_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "lsbm_test_parse_cpulist": (_int, [ctypes.c_char_p, _vp, _int]),
    "lsbm_test_cgroup_quota": (_int, [ctypes.c_char_p]),
    "lsbm_test_cgroup_quota_of": (_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "lsbm_test_pool_helpers": (_int, [_int, _int, _int]),
    "lsbm_test_locked_ranges": (_int, []),
    "lsbm_test_locks_taken": (ctypes.c_long, []),
    "lsbm_test_session_count": (_int, [_int]),
    "lsbm_test_pinned_bytes": (ctypes.c_ulonglong, [_int]),
    "lsbm_test_pool_overlap": (_int, [_int, _int, _int, _int, _vp]),
    "lsbm_test_host_pinned": (_int, [_vp, _sz]),
    "lsbm_test_host_copy": (_int, [_vp, _vp, _sz, _int]),
    "lsbm_test_pool_stress": (_int, [_int, _int, _int]),
    "lsbm_test_zero_copy_max_mb": (_int, [_int]),
    # include/lsbm_bloom.h
    "lsbm_bloom_hash": (_u32, [_vp, _sz, _u32]),
    "lsbm_bloom_filter_bytes": (_u64, [_u64, _int]),
    "lsbm_bloom_k": (_u32, [_int]),
    "lsbm_bloom_k_probe": (_u64, [_int, _int]),
    "lsbm_bloom_build_dev": (_int, [_vp, _vp, _u32, _vp, _vp, _u64, _int, _vp, _vp]),
    "lsbm_bloom_may_match_dev": (_int, [_vp, _vp, _vp, _vp, _u32, _u64, _int, _int, _vp, _vp,
                                        _vp]),
    "lsbm_filter_block_may_match_dev": (_int, [_vp, _vp, _vp, _vp, _vp, _u32, _u64, _int, _int,
                                               _vp, _vp, _vp]),
    "lsbm_snappy_max_compressed_length": (_u64, [_u64]),
    "lsbm_snappy_compress_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _vp]),
    "lsbm_snappy_uncompressed_length_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _vp]),
    "lsbm_snappy_uncompress_dev": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _vp, _vp]),
}

_lib = None


class LsbmError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__(f"{what} failed with status {code}: {last_error()}")


def lib():
    """The loaded product library (raises if it is not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: the HIP extension has not been built "
                "(run __graft_entry__.build() or make -C lsbm_amd/csrc). "
                "There is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("LSBM_LIB_PATH") and not hasattr(handle, name):
                continue  # (an older build for an A/B: only the symbols it has)
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def last_error():
    if _lib is None:
        return ""
    return (_lib.lsbm_crc32c_last_error() or b"").decode(errors="replace")


def check(rc, what):
    if rc != LSBM_OK:
        raise LsbmError(rc, what)
    return rc
