"""Shared fixtures.  `-m gpu` tests need a HIP device; everything else runs on CPU.

The oracle (oracle/liboracle_crc32c.so, a plain-C restatement of lsbm's
util/crc32c.cc) is test infrastructure: it is loaded here only as the checker.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(TESTS)
sys.path.insert(0, REPO)
sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")


class Oracle:
    """ctypes view of oracle/liboracle_crc32c.so."""

    def __init__(self, path):
        lib = ctypes.CDLL(path)
        u32, u64, vp, sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t
        lib.oracle_extend.restype = u32
        lib.oracle_extend.argtypes = [u32, vp, sz]
        lib.oracle_mask.restype = u32
        lib.oracle_mask.argtypes = [u32]
        lib.oracle_unmask.restype = u32
        lib.oracle_unmask.argtypes = [u32]
        lib.oracle_batch_offsets.restype = None
        lib.oracle_batch_offsets.argtypes = [vp, vp, u64, vp, vp, ctypes.c_int]
        lib.oracle_batch_fixed.restype = None
        lib.oracle_batch_fixed.argtypes = [vp, u64, u64, u64, vp, vp, ctypes.c_int]
        lib.oracle_batch_fixed_mt.restype = ctypes.c_int
        lib.oracle_batch_fixed_mt.argtypes = [vp, u64, u64, u64, vp, ctypes.c_int]
        lib.oracle_batch_offsets_mt.restype = ctypes.c_int
        lib.oracle_batch_offsets_mt.argtypes = [vp, u64, vp, u64, vp, ctypes.c_int]
        lib.oracle_sst_trailers_mt.restype = ctypes.c_int
        lib.oracle_sst_trailers_mt.argtypes = [vp, u64, vp, vp, u64, vp, ctypes.c_int]
        lib.oracle_fill_splitmix64.restype = None
        lib.oracle_fill_splitmix64.argtypes = [vp, u64, u64, u64]
        lib.oracle_tables.restype = None
        lib.oracle_tables.argtypes = [vp]
        self.lib = lib

    def extend(self, init, data, align=0):
        data = bytes(data)
        buf = ctypes.create_string_buffer(len(data) + 64)
        base = (ctypes.addressof(buf) + 15) & ~15
        ctypes.memmove(base + align, data, len(data))
        return self.lib.oracle_extend(init & 0xFFFFFFFF, base + align, len(data))

    def value(self, data):
        return self.extend(0, data)

    def mask(self, c):
        return self.lib.oracle_mask(c & 0xFFFFFFFF)

    def unmask(self, c):
        return self.lib.oracle_unmask(c & 0xFFFFFFFF)

    def batch_offsets(self, data, offsets, init=None, masked=False):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        self.lib.oracle_batch_offsets(data.ctypes.data, offsets.ctypes.data, n,
                                      None if ini is None else ini.ctypes.data,
                                      out.ctypes.data, 1 if masked else 0)
        return out

    def batch_fixed(self, data, stride, length, n, init=None, masked=False):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.empty(n, dtype=np.uint32)
        ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        self.lib.oracle_batch_fixed(data.ctypes.data, stride, length, n,
                                    None if ini is None else ini.ctypes.data,
                                    out.ctypes.data, 1 if masked else 0)
        return out

    @staticmethod
    def threads():
        """Worker threads for the multithreaded drivers: this process's CPU
        share (a GPU box's os.cpu_count() is the whole machine's), at most 16."""
        try:
            n = len(os.sched_getaffinity(0))
        except AttributeError:
            n = os.cpu_count() or 1
        return max(1, min(16, n))

    def batch_offsets_mt(self, window, base_off, offsets):
        """CRCs of blocks [offsets[i], offsets[i+1]) - base_off of a host window
        (a uint8 numpy array holding image bytes [base_off, base_off + size))."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        assert n >= 0 and int(offsets[0]) >= base_off and int(offsets[-1]) - base_off <= window.size
        out = np.empty(max(n, 0), dtype=np.uint32)
        assert self.lib.oracle_batch_offsets_mt(window.ctypes.data, base_off, offsets.ctypes.data, n,
                                                out.ctypes.data, self.threads()) == 0
        return out

    def sst_trailers_mt(self, window, base_off, handles, types):
        """Mask(Extend(Value(block), type)) of every handle {offset, size}
        (table/table_builder.cc:243-249), over a host window as above."""
        handles = np.ascontiguousarray(handles, dtype=np.uint64)
        types = np.ascontiguousarray(types, dtype=np.uint8)
        n = types.size
        assert handles.size == 2 * n
        if n:
            ends = handles[0::2] + handles[1::2]
            assert int(handles[0::2].min()) >= base_off and int(ends.max()) - base_off <= window.size
        out = np.empty(n, dtype=np.uint32)
        assert self.lib.oracle_sst_trailers_mt(window.ctypes.data, base_off, handles.ctypes.data,
                                               types.ctypes.data, n, out.ctypes.data, self.threads()) == 0
        return out

    def fill_splitmix64(self, byte_off, nbytes, seed):
        out = np.empty(nbytes, dtype=np.uint8)
        self.lib.oracle_fill_splitmix64(out.ctypes.data, byte_off, nbytes, seed)
        return out


class SnappyOracle:
    """ctypes view of oracle/liboracle_snappy.so (libsnappy's raw format and
    compressor restated in C, pinned to the libsnappy inside pyarrow)."""

    def __init__(self, path):
        lib = ctypes.CDLL(path)
        u32, u64, vp, i = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
        lib.so_max_compressed_length.restype = u64
        lib.so_max_compressed_length.argtypes = [u64]
        lib.so_get_uncompressed_length.restype = i
        lib.so_get_uncompressed_length.argtypes = [vp, u64, ctypes.POINTER(u32)]
        lib.so_uncompress.restype = i
        lib.so_uncompress.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64)]
        lib.so_compress.restype = u64
        lib.so_compress.argtypes = [vp, u32, vp]
        lib.so_compress_batch.restype = None
        lib.so_compress_batch.argtypes = [vp, vp, u64, vp, vp, vp]
        lib.so_uncompress_batch.restype = u64
        lib.so_uncompress_batch.argtypes = [vp, vp, u64, vp, vp, vp]
        self.lib = lib

    def max_compressed_length(self, n):
        return self.lib.so_max_compressed_length(n)

    def uncompressed_length(self, c):
        """(ok, ulength) of snappy::GetUncompressedLength."""
        b = np.frombuffer(bytes(c) + b"\0", np.uint8)
        v = ctypes.c_uint32(0)
        ok = self.lib.so_get_uncompressed_length(b.ctypes.data, len(c), ctypes.byref(v))
        return bool(ok), v.value if ok else 0

    def compress(self, d):
        d = bytes(d)
        src = np.frombuffer(d + b"\0", np.uint8)
        out = np.zeros(self.max_compressed_length(len(d)) + 8, np.uint8)
        n = self.lib.so_compress(src.ctypes.data, len(d), out.ctypes.data)
        return out[:n].tobytes()

    def uncompress(self, c, cap=None):
        """(ok, output) of snappy::RawUncompress."""
        c = bytes(c)
        ok, ulen = self.uncompressed_length(c)
        if not ok:
            return False, b""
        cap = ulen if cap is None else cap
        src = np.frombuffer(c + b"\0", np.uint8)
        out = np.zeros(max(cap, 1), np.uint8)
        got = ctypes.c_uint64(0)
        ok = self.lib.so_uncompress(src.ctypes.data, len(c), out.ctypes.data, cap, ctypes.byref(got))
        return (True, out[:got.value].tobytes()) if ok else (False, b"")


class BloomOracle:
    """ctypes view of oracle/liboracle_bloom.so (util/hash.cc, util/bloom.cc,
    table/filter_block.cc restated in C).  Keys are (uint8 buffer, uint64
    offsets) pairs, as in tests/golden/bloomkeys.py."""

    def __init__(self, path):
        lib = ctypes.CDLL(path)
        u32, u64, vp, sz, i = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_int)
        lib.bo_hash.restype = u32
        lib.bo_hash.argtypes = [vp, sz, u32]
        lib.bo_k_build.restype = sz
        lib.bo_k_build.argtypes = [i]
        lib.bo_k_probe.restype = sz
        lib.bo_k_probe.argtypes = [i, i]
        lib.bo_filter_bytes.restype = sz
        lib.bo_filter_bytes.argtypes = [sz, i]
        lib.bo_create_filter.restype = sz
        lib.bo_create_filter.argtypes = [vp, vp, sz, i, i, vp]
        lib.bo_key_may_match.restype = i
        lib.bo_key_may_match.argtypes = [vp, sz, i, vp, sz, i, i]
        lib.bo_filter_block_build.restype = sz
        lib.bo_filter_block_build.argtypes = [vp, vp, i, vp, vp, sz, i, vp, sz]
        lib.bo_filter_block_may_match.restype = i
        lib.bo_filter_block_may_match.argtypes = [vp, sz, u64, vp, sz, i, i, i]
        self.lib = lib

    @staticmethod
    def _b(x):
        return np.ascontiguousarray(np.frombuffer(bytes(x), np.uint8) if isinstance(x, (bytes, bytearray)) else x,
                                    dtype=np.uint8)

    def hash(self, data, seed=0xBC9F1D34):
        b = self._b(data)
        return self.lib.bo_hash(b.ctypes.data, b.size, seed & 0xFFFFFFFF)

    def filter_bytes(self, n, bits_per_key):
        return self.lib.bo_filter_bytes(n, bits_per_key)

    def create_filter(self, keys, bits_per_key, strip=0):
        b, o = self._b(keys[0]), np.ascontiguousarray(keys[1], dtype=np.uint64)
        n = o.size - 1
        out = np.zeros(self.filter_bytes(n, bits_per_key), dtype=np.uint8)
        self.lib.bo_create_filter(b.ctypes.data, o.ctypes.data, n, strip, bits_per_key,
                                  out.ctypes.data)
        return out.tobytes()

    def key_may_match(self, key, filt, bits_per_key, bloom_bits_use=15, strip=0):
        k, f = self._b(key), self._b(filt)
        return self.lib.bo_key_may_match(k.ctypes.data, k.size, strip, f.ctypes.data, f.size,
                                         bits_per_key, bloom_bits_use)

    def filter_block_build(self, keys, block_start, block_first, bits_per_key, strip=0):
        b, o = self._b(keys[0]), np.ascontiguousarray(keys[1], dtype=np.uint64)
        st = np.ascontiguousarray(block_start, dtype=np.uint64)
        fi = np.ascontiguousarray(block_first, dtype=np.uint64)
        need = self.lib.bo_filter_block_build(b.ctypes.data, o.ctypes.data, strip, st.ctypes.data,
                                              fi.ctypes.data, st.size, bits_per_key, None, 0)
        out = np.zeros(need, dtype=np.uint8)
        self.lib.bo_filter_block_build(b.ctypes.data, o.ctypes.data, strip, st.ctypes.data,
                                       fi.ctypes.data, st.size, bits_per_key, out.ctypes.data, need)
        return out.tobytes()

    def filter_block_may_match(self, block, block_offset, key, bits_per_key, bloom_bits_use=15,
                               strip=0):
        c, k = self._b(block), self._b(key)
        return self.lib.bo_filter_block_may_match(c.ctypes.data, c.size, block_offset,
                                                  k.ctypes.data, k.size, strip, bits_per_key,
                                                  bloom_bits_use)


def _build(target_dir, artefact):
    path = os.path.join(REPO, target_dir, artefact)
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.join(REPO, target_dir)], check=True,
                       stdout=subprocess.DEVNULL)
    return path


@pytest.fixture(scope="session")
def oracle():
    return Oracle(_build("oracle", "liboracle_crc32c.so"))


@pytest.fixture(scope="session")
def bloom_oracle():
    return BloomOracle(_build("oracle", "liboracle_bloom.so"))


@pytest.fixture(scope="session")
def snappy_oracle():
    return SnappyOracle(_build("oracle", "liboracle_snappy.so"))


@pytest.fixture(scope="session")
def snappy_golden():
    with open(os.path.join(TESTS, "golden", "snappy_fixture.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def bloom_golden():
    with open(os.path.join(TESTS, "golden", "bloom_fixture.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(TESTS, "golden", "crc32c_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def product_lib():
    _build("lsbm_amd/csrc", "../liblsbm_crc32c.so")
    from lsbm_amd import _lib
    return _lib.lib()


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from lsbm_amd import engine
    engine.init(0)
    return torch
