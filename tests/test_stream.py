"""GPU parity of the stream-major CRC kernel (lsbm_amd/csrc/crc32c_stream.hip).

Densely packed batches (offsets[], SSTable handles, log headers) go through
the stream kernel: rows are streamed per lane group regardless of block
boundaries, blocks that end in a row are saved and merged in lock-step, blocks
that cross a segment are summed across groups.  These cases aim at its seams:
block ends at every byte position of a row and of a chunk, several block ends
in one row (the general path), blocks that span segments, sub-pieces cut at
blocks out of order, extents that overlap, records past the image.  Every
result is compared with the oracle (oracle/crc32c_oracle.c, pinned to lsbm's
util/crc32c.cc by tests/test_oracle.py), block for block.
"""
import numpy as np
import pytest

from golden.splitmix import stream_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _stream_for_every_mode(torch_cuda):
    """Every batch the stream kernel takes goes to it here (by default only
    offsets[] batches do: lsbm_amd/csrc/crc32c_kernels.hip ragged_uses_stream)."""
    from lsbm_amd._lib import lib
    assert lib().lsbm_test_ragged_kernel(2) == 0
    yield
    assert lib().lsbm_test_ragged_kernel(0) == 0


def _dev(torch, arr, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if dtype is not None:
        t = t.view(dtype)
    return t.to("cuda")


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _dense(seed, lens, start=0, tail=16):
    offs = np.zeros(len(lens) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    offs += start
    data = stream_bytes(seed, 0, int(offs[-1]) + tail)
    return data, offs


def _check_offsets(torch, oracle, data, offs, masked=False):
    from lsbm_amd import engine
    got = _u32(engine.crc32c_batch(_dev(torch, data), _dev(torch, offs), masked=masked))
    want = oracle.batch_offsets(data, offs.astype(np.uint64), masked=masked)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first blocks {bad[:8].tolist()}"


@pytest.mark.parametrize("seed,n,lo,hi", [
    (1, 1, 0, 5000), (2, 7, 0, 5000), (3, 63, 0, 3000), (4, 64, 0, 3000), (5, 65, 0, 3000),
    (6, 4096, 0, 2600), (7, 100_000, 0, 2600), (8, 20_000, 1000, 9000), (9, 3000, 60_000, 70_000),
])
@pytest.mark.parametrize("start", [0, 5, 113])
def test_stream_dense_ragged(torch_cuda, oracle, seed, n, lo, hi, start):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    data, offs = _dense(seed + 100, lens, start)
    _check_offsets(torch_cuda, oracle, data, offs, masked=bool(seed & 1))


@pytest.mark.parametrize("seed,hi", [(11, 20), (12, 64), (13, 130), (14, 300)])
def test_stream_tiny_blocks_general_path(torch_cuda, oracle, seed, hi):
    """Many block ends per row: the general row path (flushes, window refills)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, hi + 1, size=50_000)
    lens[rng.random(lens.size) < 0.2] = 0
    data, offs = _dense(seed, lens, start=3)
    _check_offsets(torch_cuda, oracle, data, offs)


def test_stream_every_end_position(torch_cuda, oracle):
    """Block ends at every byte of a 128-B row: lengths cycle through 1..257."""
    lens = np.array([1 + (i * 37) % 257 for i in range(30_000)], dtype=np.int64)
    for start in (0, 1, 15, 16, 127):
        data, offs = _dense(21 + start, lens, start)
        _check_offsets(torch_cuda, oracle, data, offs)


def test_stream_segment_crossing_blocks(torch_cuda, oracle):
    """Blocks longer than a segment (T pieces summed over several groups), some
    longer than 512 rows (shifts past the column tables), mixed with short ones."""
    rng = np.random.default_rng(31)
    lens = np.concatenate([rng.integers(1 << 16, 3 << 20, size=24), rng.integers(0, 4000, size=200)])
    rng.shuffle(lens)
    data, offs = _dense(32, lens, start=7)
    _check_offsets(torch_cuda, oracle, data, offs)
    # one long block among tiny ones in every sub-piece
    lens = np.where(np.arange(4000) % 64 == 17, 700_000, rng.integers(0, 90, size=4000))
    data, offs = _dense(33, lens, start=9)
    _check_offsets(torch_cuda, oracle, data, offs)


@pytest.mark.parametrize("kind", ["reversed", "shuffled", "some_back"])
def test_stream_out_of_order_offsets(torch_cuda, oracle, kind):
    """Offsets that go back: the sub-pieces are cut at each such block (the
    block before reads as empty, as the units kernel clamps it)."""
    rng = np.random.default_rng(41)
    n = 20_000
    starts = np.sort(rng.integers(0, 30_000_000, size=n + 1))
    if kind == "reversed":
        offs = starts[::-1].copy()
    elif kind == "shuffled":
        offs = rng.permutation(starts)
    else:
        offs = starts.copy()
        idx = rng.choice(n, 300, replace=False)
        offs[idx] = rng.integers(0, 30_000_000, size=idx.size)
    data = stream_bytes(42, 0, int(starts.max()) + 16)
    from lsbm_amd import engine
    got = _u32(engine.crc32c_batch(_dev(torch_cuda, data), _dev(torch_cuda, offs.astype(np.int64))))
    # a block whose end lies before its start is empty (the engine's clamp)
    want = np.array([oracle.value(data[offs[i]:max(offs[i], offs[i + 1])].tobytes()) for i in range(n)],
                    dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first blocks {bad[:8].tolist()}"


def test_stream_overlapping_and_unsorted_extents(torch_cuda, oracle):
    from lsbm_amd import engine
    torch = torch_cuda
    rng = np.random.default_rng(51)
    data = stream_bytes(52, 0, 4_000_000)
    n = 30_000
    # mostly dense runs, with overlaps, gaps and backward jumps mixed in
    lens = rng.integers(0, 4000, size=n)
    st = np.zeros(n, dtype=np.int64)
    pos = 0
    for i in range(n):
        r = rng.random()
        if r < 0.02:
            pos = int(rng.integers(0, 3_900_000 - 4000))
        elif r < 0.04:
            pos = max(0, pos - int(rng.integers(1, 3000)))
        elif r < 0.06:
            pos += int(rng.integers(1, 200))
        if pos + lens[i] > data.size:
            pos = 0
        st[i] = pos
        pos += int(lens[i])
    ext = np.stack([st, lens], 1).reshape(-1).astype(np.int64)
    got = _u32(engine.crc32c_extents(_dev(torch, data), _dev(torch, ext)))
    want = np.array([oracle.value(data[s:s + l].tobytes()) for s, l in zip(st, lens)], dtype=np.uint32)
    assert np.array_equal(got, want)


def test_stream_gapped_extents(torch_cuda, oracle):
    """Ordered extents with gaps of 0-400 bytes between them (a block's start
    row after the row where the one before ends: no block open in between),
    blocks ending on row ends, and short and empty blocks after gaps."""
    from lsbm_amd import engine
    torch = torch_cuda
    rng = np.random.default_rng(91)
    n = 40_000
    lens = rng.integers(0, 3000, size=n)
    short = rng.random(n) < 0.1
    lens[short] = rng.integers(0, 130, size=int(short.sum()))
    gaps = rng.integers(0, 401, size=n)
    gaps[rng.random(n) < 0.3] = 0
    st = np.zeros(n, dtype=np.int64)
    pos = 11
    for i in range(n):
        pos += int(gaps[i])
        if i % 7 == 3:  # end this block on a row end
            pos += (-(pos + int(lens[i]))) % 128
        st[i] = pos
        pos += int(lens[i])
    data = stream_bytes(92, 0, pos + 64)
    ext = np.stack([st, lens], 1).reshape(-1).astype(np.int64)
    got = _u32(engine.crc32c_extents(_dev(torch, data), _dev(torch, ext)))
    want = np.array([oracle.value(data[s:s + l].tobytes()) for s, l in zip(st, lens)], dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first blocks {bad[:8].tolist()}"


def test_stream_verify_flags_flips(torch_cuda, oracle):
    from lsbm_amd import engine
    torch = torch_cuda
    rng = np.random.default_rng(61)
    lens = rng.integers(0, 3000, size=60_000)
    data, offs = _dense(62, lens, start=1)
    want = oracle.batch_offsets(data, offs.astype(np.uint64), masked=True)
    bad_blocks = rng.choice(np.nonzero(lens > 0)[0], 200, replace=False)
    for b in bad_blocks:
        data[offs[b] + rng.integers(0, lens[b])] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ok, nbad = engine.crc32c_verify(_dev(torch, data), _dev(torch, offs),
                                    _dev(torch, want.view(np.int32)), masked=True)
    ok = ok.cpu().numpy()
    assert int(nbad.item()) == bad_blocks.size
    assert set(np.nonzero(ok == 0)[0].tolist()) == set(bad_blocks.tolist())


def test_stream_sst_layout_all_modes(torch_cuda, oracle):
    """A table image of blocks of 0-9000 B with 5-byte trailers (and some
    index/filter-sized blocks): trailer CRCs, seal, verify, corruptions."""
    from lsbm_amd import table
    torch = torch_cuda
    rng = np.random.default_rng(71)
    sizes = np.concatenate([rng.integers(0, 9000, size=5000), rng.integers(30_000, 200_000, size=8)])
    rng.shuffle(sizes)
    handles, total = table.layout_blocks(sizes)
    img = stream_bytes(72, 0, int(total))
    types = rng.integers(0, 2, size=sizes.size).astype(np.uint8)
    d = _dev(torch, img)
    dh = _dev(torch, np.ascontiguousarray(handles, dtype=np.int64))
    dt = _dev(torch, types)
    crcs = _u32(table.trailer_crcs(d, dh, dt)[0])
    off, sz = handles[0::2], handles[1::2]
    for i in range(sizes.size):
        blk = img[off[i]:off[i] + sz[i]].tobytes() + bytes([types[i]])
        assert crcs[i] == oracle.mask(oracle.value(blk)), i
    table.seal_blocks(d, dh, dt)
    ok, nbad = table.verify_blocks(d, dh)
    assert bool(ok.all()) and int(nbad.item()) == 0
    sealed = d.cpu().numpy()
    # corrupt 40 blocks (payload, type byte or stored crc)
    bad = rng.choice(sizes.size, 40, replace=False)
    for b in bad:
        where = int(rng.integers(0, sz[b] + 5))
        sealed[off[b] + where] ^= 0x40
    ok, nbad = table.verify_blocks(_dev(torch, sealed), dh)
    assert set(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == set(bad.tolist())
    assert int(nbad.item()) == bad.size


def test_stream_log_records(torch_cuda, oracle):
    """A WAL image of records of 0-2540 B (framed by the reference rules):
    seal, dense CRCs, verify, and a flipped record."""
    import ctypes
    from golden.splitmix import printable_bytes
    from lsbm_amd import log
    from lsbm_amd._lib import lib
    torch = torch_cuda
    rng = np.random.default_rng(81)
    lens = rng.integers(0, 2541, size=20_000)
    short = rng.random(lens.size) < 0.05
    lens[short] = rng.integers(0, 40, size=int(short.sum()))
    pay = printable_bytes(82, int(lens.sum()))
    offs = np.concatenate([[0], np.cumsum(lens)])
    wimg, heads = log.layout_records(pay[offs[i]:offs[i + 1]] for i in range(lens.size))
    d = _dev(torch, wimg)
    dh = _dev(torch, heads)
    n = heads.size
    masked = torch.empty(n, dtype=torch.int32, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = lib()
    dp, hp, mp, bp, op = (ctypes.c_void_p(t.data_ptr()) for t in (d, dh, masked, nbad, ok))
    nb = ctypes.c_uint64(d.numel())
    assert L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, s) == 0
    img = d.cpu().numpy()
    plen = img[heads + 4].astype(np.int64) | (img[heads + 5].astype(np.int64) << 8)
    got = _u32(masked)
    for i in range(n):
        h = int(heads[i])
        want = oracle.mask(oracle.value(img[h + 6:h + 7 + int(plen[i])].tobytes()))
        assert got[i] == want, i
        assert int.from_bytes(img[h:h + 4].tobytes(), "little") == want, i
    assert L.lsbm_log_verify_dev(dp, nb, hp, n, op, bp, s) == 0
    assert bool(ok.all().item()) and int(nbad.item()) == 0
    bad = rng.choice(n, 25, replace=False)
    for b in bad:
        h = int(heads[b])
        img[h + 6 + int(rng.integers(0, plen[b] + 1))] ^= 0x08
    d2 = _dev(torch, img)
    nbad.zero_()
    assert L.lsbm_log_verify_dev(ctypes.c_void_p(d2.data_ptr()), nb, hp, n, op, bp, s) == 0
    assert set(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == set(bad.tolist())
    assert int(nbad.item()) == bad.size
