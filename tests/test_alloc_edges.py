"""Batches flush against the ends of fresh hipMalloc allocations.

The ragged kernels' loads must stay inside the batch's bytes: the units kernel
keeps its row loads in bounds by clamped addresses that empty `asm volatile`
pins protect from being folded (lsbm_amd/csrc/crc32c_units.h), the stream
kernel by buffer descriptors bounded to each sub-piece.  A regression there
reads past the data.  Here the image, the extent arrays and the outputs each
sit flush against the start or the end of their own allocation (sizes a
multiple of 2 MiB, so the allocation's last byte is the end of its mapping),
with idle lanes in every round: n % 8 != 0, empty blocks, batches of fewer
than 8 blocks.  Every units-kernel instantiation runs (policy 1: Out x
{offsets, extents, fixed}, Verify, SstSeal, SstVerify, SstCrc, LogSeal,
LogVerify) and every stream-kernel one (policy 2).  A stray access faults the
test instead of a user's compaction; every result is checked against the
oracle (oracle/crc32c_oracle.c).
"""
import ctypes

import numpy as np
import pytest

from golden.splitmix import printable_bytes, stream_bytes

pytestmark = pytest.mark.gpu

GRAN = 2 << 20


class Hip:
    def __init__(self):
        self.h = ctypes.CDLL("libamdhip64.so")
        self.h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.h.hipFree.argtypes = [ctypes.c_void_p]
        self.h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        self.h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        self.live = []

    def place(self, arr, at_end=True):
        """A fresh allocation of a 2 MiB multiple holding `arr`'s bytes flush
        against its end (or start); returns the device address of the bytes."""
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        size = max(GRAN, -(-b.size // GRAN) * GRAN)
        p = ctypes.c_void_p()
        assert self.h.hipMalloc(ctypes.byref(p), size) == 0
        self.live.append(p.value)
        assert self.h.hipMemset(p.value, 0xA5, size) == 0
        addr = p.value + (size - b.size if at_end else 0)
        if b.size:
            assert self.h.hipMemcpy(addr, b.ctypes.data, b.size, 1) == 0
        return addr

    def out(self, nbytes, at_end=True):
        return self.place(np.zeros(nbytes, dtype=np.uint8), at_end)

    def get(self, addr, nbytes, dtype):
        b = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            assert self.h.hipMemcpy(b.ctypes.data, addr, nbytes, 2) == 0
        return b.view(dtype)

    def free(self):
        for p in self.live:
            self.h.hipFree(p)
        self.live = []


@pytest.fixture
def hip(torch_cuda):
    h = Hip()
    yield h
    h.free()


@pytest.fixture(params=[1, 2], ids=["units", "stream"])
def policy(request, torch_cuda):
    from lsbm_amd._lib import lib
    assert lib().lsbm_test_ragged_kernel(request.param) == 0
    yield request.param
    assert lib().lsbm_test_ragged_kernel(0) == 0


def _lens(rng, n):
    lens = rng.integers(0, 700, size=n)
    lens[rng.random(n) < 0.2] = 0
    if n > 3:
        lens[1] = 4096
        lens[2] = 0
    return lens


def _sync():
    import torch
    torch.cuda.synchronize()


CASES = [(1, True), (7, False), (13, True), (1001, False), (4099, True)]


@pytest.mark.parametrize("n,at_end", CASES)
def test_offsets_extents_verify_at_allocation_edges(hip, policy, oracle, n, at_end):
    from lsbm_amd._lib import lib
    L = lib()
    rng = np.random.default_rng(n)
    lens = _lens(rng, n)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    data = stream_bytes(n + 7, 0, int(offs[-1]))
    base = hip.place(data, at_end)
    do = hip.place(offs, at_end)
    want = oracle.batch_offsets(data, offs.astype(np.uint64))
    # crc32c_batch (Out, offsets)
    out = hip.out(4 * n, at_end)
    assert L.lsbm_crc32c_batch_dev(base, do, n, None, out, 0, None) == 0
    _sync()
    assert np.array_equal(hip.get(out, 4 * n, np.uint32), want)
    # extents (Out, {offset, length})
    ext = np.stack([offs[:-1], lens], 1).reshape(-1).astype(np.int64)
    de = hip.place(ext, at_end)
    out2 = hip.out(4 * n, at_end)
    assert L.lsbm_crc32c_extents_dev(base, de, n, None, out2, 0, None) == 0
    _sync()
    assert np.array_equal(hip.get(out2, 4 * n, np.uint32), want)
    # verify (offsets) against the CRCs, one flipped expectation
    exp = want.copy()
    exp[n // 2] ^= 1
    dx = hip.place(exp, at_end)
    ok = hip.out(n, at_end)
    nbad = hip.out(4, at_end)
    assert L.lsbm_crc32c_verify_dev(base, do, n, None, dx, ok, nbad, 0, None) == 0
    _sync()
    okv = hip.get(ok, n, np.uint8)
    assert okv[n // 2] == 0 and int(okv.sum()) == n - 1
    assert int(hip.get(nbad, 4, np.uint32)[0]) == 1


@pytest.mark.parametrize("n,at_end", CASES)
def test_fixed_ragged_geometry_at_allocation_edges(hip, policy, oracle, n, at_end):
    """lsbm_crc32c_fixed_dev off its fast path (len not a multiple of 128, odd
    stride): the units kernel's fixed-stride extents."""
    from lsbm_amd._lib import lib
    L = lib()
    length, stride = 100 + n % 50, 163
    total = (n - 1) * stride + length
    data = stream_bytes(n + 11, 0, total)
    base = hip.place(data, at_end)
    out = hip.out(4 * n, at_end)
    assert L.lsbm_crc32c_fixed_dev(base, stride, length, n, None, out, 0, None) == 0
    _sync()
    assert np.array_equal(hip.get(out, 4 * n, np.uint32), oracle.batch_fixed(data, stride, length, n))


@pytest.mark.parametrize("n,at_end", CASES)
def test_sst_modes_at_allocation_edges(hip, policy, oracle, n, at_end):
    from lsbm_amd import table
    from lsbm_amd._lib import lib
    L = lib()
    rng = np.random.default_rng(100 + n)
    sizes = _lens(rng, n)
    handles, total = table.layout_blocks(sizes)
    img = printable_bytes(n + 13, total).copy()
    types = rng.integers(0, 2, size=n).astype(np.uint8)
    base = hip.place(img, at_end)
    dh = hip.place(handles.astype(np.int64), at_end)
    dt = hip.place(types, at_end)
    off, sz = handles[0::2], handles[1::2]
    want = np.array([oracle.mask(oracle.extend(oracle.value(img[o:o + s].tobytes()), bytes([t])))
                     for o, s, t in zip(off, sz, types)], dtype=np.uint32)
    # dense trailer CRCs (SstCrc)
    crcs = hip.out(4 * n, at_end)
    nbad = hip.out(4, at_end)
    assert L.lsbm_sst_trailer_crcs_dev(base, total, dh, dt, n, crcs, nbad, None) == 0
    _sync()
    assert np.array_equal(hip.get(crcs, 4 * n, np.uint32), want)
    # seal in place (one pass below 131072 blocks: SstSeal)
    assert L.lsbm_sst_seal_dev(base, total, dh, dt, n, nbad, None) == 0
    _sync()
    sealed = hip.get(base, total, np.uint8)
    for i in range(n):
        o, s = int(off[i]), int(sz[i])
        assert sealed[o + s] == types[i]
        assert int.from_bytes(sealed[o + s + 1:o + s + 5].tobytes(), "little") == want[i]
    assert int(hip.get(nbad, 4, np.uint32)[0]) == 0
    # verify (SstVerify): all ok, then one corrupted block
    ok = hip.out(n, at_end)
    assert L.lsbm_sst_verify_dev(base, total, dh, n, ok, nbad, None) == 0
    _sync()
    assert int(hip.get(ok, n, np.uint8).sum()) == n
    b = n - 1
    flip = np.array([sealed[int(off[b]) + int(sz[b])] ^ 0x40], dtype=np.uint8)
    hip.h.hipMemcpy(base + int(off[b]) + int(sz[b]), flip.ctypes.data, 1, 1)
    assert L.lsbm_sst_verify_dev(base, total, dh, n, ok, nbad, None) == 0
    _sync()
    okv = hip.get(ok, n, np.uint8)
    assert okv[b] == 0 and int(okv.sum()) == n - 1


@pytest.mark.parametrize("n,at_end", CASES)
def test_log_modes_at_allocation_edges(hip, policy, oracle, n, at_end):
    from lsbm_amd import log
    from lsbm_amd._lib import lib
    L = lib()
    rng = np.random.default_rng(200 + n)
    lens = _lens(rng, n)
    pay = printable_bytes(n + 17, int(lens.sum()))
    po = np.concatenate([[0], np.cumsum(lens)])
    img, heads = log.layout_records(pay[po[i]:po[i + 1]] for i in range(n))
    m = heads.size
    base = hip.place(img, at_end)
    dh = hip.place(heads.astype(np.int64), at_end)
    plen = img[heads + 4].astype(np.int64) | (img[heads + 5].astype(np.int64) << 8)
    want = np.array([oracle.mask(oracle.value(img[h + 6:h + 7 + int(p)].tobytes()))
                     for h, p in zip(heads, plen)], dtype=np.uint32)
    crcs = hip.out(4 * m, at_end)
    nbad = hip.out(4, at_end)
    assert L.lsbm_log_crcs_dev(base, img.size, dh, m, crcs, nbad, None) == 0
    _sync()
    assert np.array_equal(hip.get(crcs, 4 * m, np.uint32), want)
    out = hip.out(4 * m, at_end)
    assert L.lsbm_log_seal_dev(base, img.size, dh, m, out, nbad, None) == 0
    _sync()
    assert np.array_equal(hip.get(out, 4 * m, np.uint32), want)
    sealed = hip.get(base, img.size, np.uint8)
    for h, w in zip(heads, want):
        assert int.from_bytes(sealed[h:h + 4].tobytes(), "little") == w
    ok = hip.out(m, at_end)
    assert L.lsbm_log_verify_dev(base, img.size, dh, m, ok, nbad, None) == 0
    _sync()
    assert int(hip.get(ok, m, np.uint8).sum()) == m
    assert int(hip.get(nbad, 4, np.uint32)[0]) == 0
