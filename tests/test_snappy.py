"""Snappy block codec: oracle pinning (CPU) and GPU parity (`-m gpu`).

The reference compresses SSTable blocks through port::Snappy_* (port/port_posix.h:119-150
-> libsnappy RawCompress / GetUncompressedLength / RawUncompress), from
TableBuilder::WriteBlock (table/table_builder.cc:181-193: keep the compressed form
only if it saves at least 1/8) and ReadBlock (table/format.cc:124-141:
"corrupted compressed block contents" when either call fails).  libsnappy is a
third-party dependency absent from /root/reference; the oracle
(oracle/snappy_oracle.c) is pinned to the libsnappy inside pyarrow through
tests/golden/snappy_fixture.json (tests/golden/make_snappy_fixture.py).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from snappy_inputs import block, mutations, varint32  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()


def crafted_bytes(name, rec):
    if rec["hex"] is not None:
        return bytes.fromhex(rec["hex"])
    assert name == "literal_ext3"
    return varint32(70000) + bytes([62 << 2]) + (69999).to_bytes(3, "little") + b"z" * 70000


# ---------------------------------------------------------------- oracle pinning (CPU)

def test_oracle_compress_matches_libsnappy(snappy_oracle, snappy_golden):
    for cs in snappy_golden["cases"]:
        d = block(cs["kind"], cs["n"], cs["seed"])
        c = snappy_oracle.compress(d)
        assert len(c) == cs["clen"] and sha(c) == cs["csha"], (cs["kind"], cs["n"])
        assert c[:24].hex() == cs["head"]
        assert (len(c) < cs["n"] - cs["n"] // 8) == cs["store_compressed"]
        assert snappy_oracle.uncompress(c) == (True, d)


def test_oracle_uncompress_corruptions_match_libsnappy(snappy_oracle, snappy_golden):
    cases = snappy_golden["cases"]
    by_case = {}
    for rec in snappy_golden["corrupt"]:
        by_case.setdefault(rec["case"], []).append(rec)
    n_ok = 0
    for i, recs in by_case.items():
        cs = cases[i]
        c = snappy_oracle.compress(block(cs["kind"], cs["n"], cs["seed"]))
        muts = dict(mutations(c, 7000 + i))
        for rec in recs:
            ok, out = snappy_oracle.uncompress(muts[rec["mutation"]])
            assert ok == rec["ok"], (i, rec["mutation"])
            if ok:
                n_ok += 1
                assert len(out) == rec["out_len"] and sha(out) == rec["out_sha"]
    assert 0 < n_ok < len(snappy_golden["corrupt"])


def test_oracle_crafted_streams_match_libsnappy(snappy_oracle, snappy_golden):
    for rec in snappy_golden["crafted"]:
        ok, out = snappy_oracle.uncompress(crafted_bytes(rec["name"], rec))
        assert ok == rec["ok"], rec["name"]
        if ok:
            assert len(out) == rec["out_len"] and sha(out) == rec["out_sha"], rec["name"]


def test_oracle_length_and_bounds(snappy_oracle):
    assert snappy_oracle.max_compressed_length(4096) == 32 + 4096 + 4096 // 6
    assert snappy_oracle.uncompressed_length(varint32(300)) == (True, 300)
    assert snappy_oracle.uncompressed_length(b"") == (False, 0)
    assert snappy_oracle.uncompressed_length(bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F])) == (True, 0xFFFFFFFF)
    # a capacity below the preamble length fails, like an undersized output buffer
    c = snappy_oracle.compress(b"abc" * 100)
    assert snappy_oracle.uncompress(c, cap=299) == (False, b"")


def test_lane_walk_model_matches_oracle(snappy_oracle, snappy_golden):
    """The decoder's lane-parallel window walk (decode_lanes, restated in
    tools/snappy_lanes_model.py) accepts and rejects exactly what the oracle
    does, and writes the same bytes, on a subset of the fixture blocks, all
    their corruptions and the crafted streams (the whole set: run the tool)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from snappy_lanes_model import decode_lanes
    n = 0
    streams = []
    for k, cs in enumerate(snappy_golden["cases"][:24:3]):
        if cs["n"] > 0x3000:
            continue
        c = snappy_oracle.compress(block(cs["kind"], cs["n"], cs["seed"]))
        streams.append(c)
        streams.extend(m for _, m in mutations(c, 7000 + 3 * k))
    streams.extend(crafted_bytes(r["name"], r) for r in snappy_golden["crafted"] if r["name"] != "literal_ext3")
    for st in streams:
        okp, ulen = snappy_oracle.uncompressed_length(st)
        if not okp or ulen > 0x3000:
            continue
        i = 0
        while st[i] >= 128:
            i += 1
        assert decode_lanes(st[i + 1:], ulen) == snappy_oracle.uncompress(st)
        n += 1
    assert n >= 40


def test_snappy_entry_points_fail_loudly_without_device(product_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from lsbm_amd import _lib
    L = _lib.lib()
    z = np.zeros(16, dtype=np.uint64)
    buf = np.zeros(64, dtype=np.uint8)
    assert L.lsbm_snappy_max_compressed_length(4096) == 32 + 4096 + 4096 // 6
    assert L.lsbm_snappy_compress_dev(buf.ctypes.data, z.ctypes.data, 1, buf.ctypes.data,
                                      z.ctypes.data, z.ctypes.data, None) == _lib.LSBM_ERR_NO_DEVICE
    assert L.lsbm_snappy_uncompress_dev(buf.ctypes.data, z.ctypes.data, 1, buf.ctypes.data,
                                        z.ctypes.data, buf.ctypes.data, None, None) == \
        _lib.LSBM_ERR_NO_DEVICE
    assert L.lsbm_snappy_uncompressed_length_dev(buf.ctypes.data, z.ctypes.data, 1, z.ctypes.data,
                                                 buf.ctypes.data, None) == _lib.LSBM_ERR_NO_DEVICE
    assert L.lsbm_snappy_uncompress_dev(None, None, 1, None, None, None, None, None) == \
        _lib.LSBM_ERR_INVALID
    assert L.lsbm_snappy_compress_dev(None, None, 0, None, None, None, None) == _lib.LSBM_OK


# ---------------------------------------------------------------- GPU

def _pack(blocks):
    offs = np.zeros(len(blocks) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in blocks])
    data = np.frombuffer(b"".join(blocks) + b"\0", dtype=np.uint8)
    return data, offs


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def gpu_compress(torch, blocks):
    from lsbm_amd import snappy
    data, offs = _pack(blocks)
    out, oo, ol = snappy.compress(_dev(torch, data), _dev(torch, offs))
    torch.cuda.synchronize()
    out, oo, ol = out.cpu().numpy(), oo.cpu().numpy(), ol.cpu().numpy()
    return [out[oo[i]:oo[i] + ol[i]].tobytes() for i in range(len(blocks))]


def gpu_uncompress(torch, streams, caps=None):
    """[(ok, output)] of the GPU RawUncompress; caps = output capacity per block
    (default: the oracle-independent preamble lengths from the GPU)."""
    from lsbm_amd import snappy
    data, offs = _pack(streams)
    d, o = _dev(torch, data), _dev(torch, offs)
    if caps is None:
        ulen, lok = snappy.uncompressed_length(d, o)
        caps = np.where(lok.cpu().numpy() == 1, ulen.cpu().numpy(), 0)
    oo = np.zeros(len(streams) + 1, dtype=np.int64)
    oo[1:] = np.cumsum(caps)
    out, _, ok, n_bad = snappy.uncompress(d, o, out_offsets=_dev(torch, oo))
    torch.cuda.synchronize()
    out, ok = out.cpu().numpy(), ok.cpu().numpy()
    assert int(n_bad.item()) == int((ok == 0).sum())
    return [(bool(ok[i]), out[oo[i]:oo[i + 1]].tobytes() if ok[i] else b"") for i in range(len(streams))]


@pytest.mark.gpu
def test_gpu_compress_matches_libsnappy(torch_cuda, snappy_golden):
    cases = snappy_golden["cases"]
    blocks = [block(c["kind"], c["n"], c["seed"]) for c in cases]
    got = gpu_compress(torch_cuda, blocks)
    for c, g in zip(cases, got):
        assert len(g) == c["clen"] and sha(g) == c["csha"], (c["kind"], c["n"])


@pytest.mark.gpu
def test_gpu_uncompress_roundtrip_fixture(torch_cuda, snappy_oracle, snappy_golden):
    cases = snappy_golden["cases"]
    blocks = [block(c["kind"], c["n"], c["seed"]) for c in cases]
    comp = [snappy_oracle.compress(b) for b in blocks]
    for (ok, out), b in zip(gpu_uncompress(torch_cuda, comp), blocks):
        assert ok and out == b


@pytest.mark.gpu
def test_gpu_uncompress_corruptions_and_crafted(torch_cuda, snappy_oracle, snappy_golden):
    cases = snappy_golden["cases"]
    streams, expect = [], []
    for rec in snappy_golden["corrupt"]:
        cs = cases[rec["case"]]
        c = snappy_oracle.compress(block(cs["kind"], cs["n"], cs["seed"]))
        streams.append(dict(mutations(c, 7000 + rec["case"]))[rec["mutation"]])
        expect.append(rec)
    for rec in snappy_golden["crafted"]:
        streams.append(crafted_bytes(rec["name"], rec))
        expect.append(rec)
    # capacity = the preamble length when it is small, else nothing (huge
    # preambles from corruption would need GiBs; the oracle then fails too)
    caps = []
    for s in streams:
        ok, ulen = snappy_oracle.uncompressed_length(s)
        caps.append(ulen if ok and ulen <= (1 << 20) else 0)
    got = gpu_uncompress(torch_cuda, streams, caps=np.array(caps, dtype=np.int64))
    for s, cap, rec, (ok, out) in zip(streams, caps, expect, got):
        ook, oout = snappy_oracle.uncompress(s, cap=cap)
        assert ok == ook, rec
        assert out == oout
        ok_ulen = snappy_oracle.uncompressed_length(s)
        if ok_ulen[0] and ok_ulen[1] <= (1 << 20):
            assert ok == rec["ok"], rec
            if ok:
                assert sha(out) == rec["out_sha"]


@pytest.mark.gpu
def test_gpu_uncompressed_length(torch_cuda, snappy_oracle):
    from lsbm_amd import snappy
    streams = [b"", b"\x00", varint32(300), varint32(0xFFFFFFFF), bytes([0x80] * 4 + [0x10]),
               bytes([0x80, 0x80]), snappy_oracle.compress(b"x" * 5000)]
    data, offs = _pack(streams)
    ulen, ok = snappy.uncompressed_length(_dev(torch_cuda, data), _dev(torch_cuda, offs))
    got = list(zip(ok.cpu().numpy().tolist(), ulen.cpu().numpy().tolist()))
    want = [snappy_oracle.uncompressed_length(s) for s in streams]
    assert [(bool(a), b) for a, b in got] == want


@pytest.mark.gpu
def test_gpu_uncompress_huge_preamble_among_good_blocks(torch_cuda, snappy_oracle):
    """A preamble claiming 4 GiB (more than snappy's 22x expansion of its
    compressed bytes allows) gets no window and fails alone; the good blocks
    around it decode (lsbm_amd/snappy.py MAX_EXPANSION)."""
    from lsbm_amd import snappy
    good = [block("records", 4117 + i, 60000 + i) for i in range(6)]
    streams = [snappy_oracle.compress(b) for b in good]
    streams.insert(3, varint32(0xFFFFFFFF) + b"a" * 40)
    data, offs = _pack(streams)
    out, out_offsets, ok, n_bad = snappy.uncompress(_dev(torch_cuda, data), _dev(torch_cuda, offs))
    assert out.numel() < (1 << 20)
    okh = ok.cpu().numpy().tolist()
    assert okh == [1, 1, 1, 0, 1, 1, 1] and int(n_bad.item()) == 1
    oo = out_offsets.cpu().numpy()
    outh = out.cpu().numpy()
    for j, i in enumerate([0, 1, 2, 4, 5, 6]):
        assert outh[oo[i]:oo[i + 1]].tobytes() == good[j]


@pytest.mark.gpu
def test_gpu_capacity_below_preamble_fails(torch_cuda, snappy_oracle):
    c = snappy_oracle.compress(b"abcd" * 1000)
    got = gpu_uncompress(torch_cuda, [c, c], caps=np.array([3999, 4000], dtype=np.int64))
    assert got[0] == (False, b"") and got[1] == (True, b"abcd" * 1000)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["records", "random", "printable"])
def test_gpu_sstable_sized_batch(torch_cuda, snappy_oracle, kind):
    """5,000 SSTable-sized blocks (4,117-4,122 B, the db_bench data block
    sizes): every compressed block checked against the oracle; GPU round trip."""
    torch = torch_cuda
    rng = np.random.default_rng(42)
    lens = rng.integers(4117, 4123, 5000)
    blocks = [block(kind, int(n), 50000 + i) for i, n in enumerate(lens)]
    got = gpu_compress(torch, blocks)
    for i in range(0, len(blocks)):
        assert got[i] == snappy_oracle.compress(blocks[i]), i
    back = gpu_uncompress(torch, got)
    assert all(ok and out == b for (ok, out), b in zip(back, blocks))
