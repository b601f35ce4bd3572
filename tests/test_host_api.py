"""CPU-side checks of the product library and its C ABI (no GPU compute).

* liblsbm_crc32c.so loads and exports every function include/lsbm_crc32c.h
  declares, plus the reference's mangled leveldb::crc32c::Extend;
* the scalar API (include/util/crc32c.h) matches the reference golden vectors;
* a C++ program written against util/crc32c.h links unchanged;
* batch entry points fail loudly (LSBM_ERR_*) instead of computing on the CPU
  when no device is present.
"""
import os
import re
import subprocess

import ctypes

import numpy as np
import pytest

from golden.splitmix import printable_bytes, stream_bytes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    """Every C function the C-ABI headers (include/lsbm_*.h) declare."""
    names = set()
    for h in ("lsbm_crc32c.h", "lsbm_bloom.h", "lsbm_snappy.h"):
        text = open(os.path.join(REPO, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(lsbm_\w+)\s*\(", text))
    return sorted(names)


def test_exports_every_declared_symbol(product_lib):
    names = declared_functions()
    assert len(names) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", product_lib._name],
                         capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if " T " in line)
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" in exported  # util/crc32c.h:17
    assert "_ZN7leveldb4HashEPKcmj" in exported  # util/hash.h:15
    from lsbm_amd import _lib
    assert sorted(_lib.SIGNATURES) == names


def test_scalar_api_matches_reference(product_lib, golden):
    from lsbm_amd import crc32c
    for k in golden["kat"]:
        assert crc32c.value(bytes.fromhex(k["hex"])) == k["value"]
    for c in golden["random"]:
        data = stream_bytes(c["seed"], 0, c["len"]).tobytes()
        v = crc32c.extend(c["init"], data)
        assert v == c["value"], c
        assert crc32c.mask(v) == c["mask"]
        assert crc32c.unmask(c["mask"]) == v
    for b in golden["sst_blocks"]:
        blk = printable_bytes(b["seed"], b["len"]).tobytes()
        assert crc32c.extend(crc32c.value(blk), bytes([b["type"]])) == b["crc"]
    assert crc32c.MASK_DELTA == 0xA282EAD8


def _aligned_copy(data, align):
    """data at an address that is `align` mod 16 (the buffer stays alive with it)."""
    buf = ctypes.create_string_buffer(len(data) + 64)
    base = (ctypes.addressof(buf) + 15) & ~15
    ctypes.memmove(base + align, data, len(data))
    return buf, base + align


def test_scalar_extend_at_golden_alignments(product_lib, golden):
    """The golden cases at their recorded alignment (tests/golden/make_golden.py
    placed each case's bytes `align` bytes past a 64-B boundary for the
    reference's Extend; here past a 16-B one, the same mod 8 and 16): through
    lsbm_crc32c_extend and through the C++ symbol
    the unchanged table/ and log code links (its SSE4.2 path runs a byte-wise
    prologue up to the first 8-B boundary, lsbm_amd/csrc/crc32c_host.cc)."""
    L = product_lib
    cxx = getattr(L, "_ZN7leveldb6crc32c6ExtendEjPKcm")
    cxx.restype = ctypes.c_uint32
    cxx.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    aligns = set()
    for c in golden["random"]:
        data = stream_bytes(c["seed"], 0, c["len"]).tobytes()
        buf, p = _aligned_copy(data, c["align"])
        aligns.add(c["align"])
        assert L.lsbm_crc32c_extend(c["init"], ctypes.c_void_p(p), len(data)) == c["value"], c
        assert cxx(c["init"], p, len(data)) == c["value"], c
    assert len(aligns) >= 8  # the golden set spans the alignments


def test_scalar_extend_every_alignment(product_lib, oracle):
    """Every start alignment mod 16 and short / word-straddling lengths."""
    L = product_lib
    rng = np.random.default_rng(9)
    for n in [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33, 63, 65, 127, 255, 4096, 4101]:
        data = stream_bytes(int(rng.integers(0, 2**62)), 0, n).tobytes()
        init = int(rng.integers(0, 2**32))
        want = oracle.extend(init, data)
        for align in range(16):
            buf, p = _aligned_copy(data, align)
            assert L.lsbm_crc32c_extend(init, ctypes.c_void_p(p), n) == want, (n, align)


def test_scalar_api_matches_oracle_sizes(product_lib, oracle):
    from lsbm_amd import crc32c
    rng = np.random.default_rng(5)
    for n in list(range(0, 80)) + [1023, 1024, 3071, 3072, 3073, 6144, 9217, 100000]:
        data = stream_bytes(int(rng.integers(0, 2**62)), 0, n).tobytes()
        init = int(rng.integers(0, 2**32))
        assert crc32c.extend(init, data) == oracle.extend(init, data)


def test_cpp_links_unchanged(product_lib, tmp_path):
    exe = tmp_path / "link_test"
    libdir = os.path.join(REPO, "lsbm_amd")
    subprocess.run(["g++", "-O2", "-std=c++11", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "link_test.cc"), "-L", libdir,
                    "-llsbm_crc32c", "-Wl,-rpath," + libdir, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


def test_batch_entry_points_fail_loudly_without_device(product_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from lsbm_amd import _lib
    L = _lib.lib()
    out = np.zeros(4, dtype=np.uint32)
    data = np.zeros(4096 * 4, dtype=np.uint8)
    # a host pointer is not a device pointer, but with no device the call must
    # refuse before touching anything
    rc = L.lsbm_crc32c_fixed_dev(data.ctypes.data, 4096, 4096, 4, None, out.ctypes.data, 0, None)
    assert rc == _lib.LSBM_ERR_NO_DEVICE
    offs = np.array([0, 10, 20], dtype=np.uint64)
    rc = L.lsbm_crc32c_batch_host(0, data.ctypes.data, offs.ctypes.data, 2, None,
                                  out.ctypes.data, 0)
    assert rc == _lib.LSBM_ERR_NO_DEVICE
    assert L.lsbm_crc32c_init(0) == _lib.LSBM_ERR_NO_DEVICE
    assert np.all(out == 0)


def test_argument_validation(product_lib):
    from lsbm_amd import _lib
    L = _lib.lib()
    out = np.zeros(4, dtype=np.uint32)
    assert L.lsbm_crc32c_fixed_dev(None, 4096, 4096, 4, None, out.ctypes.data, 0, None) == \
        _lib.LSBM_ERR_INVALID
    assert L.lsbm_crc32c_batch_dev(None, None, 4, None, None, 0, None) == _lib.LSBM_ERR_INVALID
    assert L.lsbm_crc32c_fixed_dev(None, 0, 0, 0, None, None, 0, None) == _lib.LSBM_OK  # n == 0
    assert L.lsbm_crc32c_version().startswith(b"lsbm-crc32c")
