"""Pin the oracle (oracle/crc32c_oracle.c) to the reference's golden vectors.

tests/golden/crc32c_golden.json was produced by tests/golden/make_golden.py
from lsbm's own util/crc32c.cc (compiled from /root/reference by
oracle/Makefile).  Every vector must match bit for bit.
"""
import numpy as np

from golden.splitmix import printable_bytes, stream_bytes


def test_kat_rfc3720(oracle, golden):
    for k in golden["kat"]:
        data = bytes.fromhex(k["hex"])
        assert oracle.value(data) == k["value"], k["name"]
        assert oracle.mask(oracle.value(data)) == k["mask"], k["name"]
    # RFC 3720 B.4 literal values
    names = {k["name"]: k["value"] for k in golden["kat"]}
    assert names["zeros32"] == 0x8A9136AA
    assert names["ones32"] == 0x62A8AB43
    assert names["inc32"] == 0x46DD794E
    assert names["dec32"] == 0x113FDB5C
    assert names["123456789"] == 0xE3069283


def test_extend_and_mask_chain(oracle, golden):
    c = golden["extend_chain"]
    a = oracle.value(c["a"].encode())
    assert a == c["value_a"]
    assert oracle.extend(a, c["b"].encode()) == c["extend"]
    assert oracle.value((c["a"] + c["b"]).encode()) == c["extend"]
    m = golden["mask_chain"]
    assert oracle.mask(m["crc"]) == m["mask"]
    assert oracle.mask(oracle.mask(m["crc"])) == m["mask2"]
    assert oracle.unmask(oracle.mask(m["crc"])) == m["crc"]


def test_random_cases_all_alignments(oracle, golden):
    for c in golden["random"]:
        data = stream_bytes(c["seed"], 0, c["len"]).tobytes()
        v = oracle.extend(c["init"], data, c["align"])
        assert v == c["value"], c
        assert oracle.mask(v) == c["mask"]


def test_sst_trailers(oracle, golden):
    for b in golden["sst_blocks"]:
        blk = printable_bytes(b["seed"], b["len"]).tobytes()
        crc = oracle.extend(oracle.value(blk), bytes([b["type"]]))
        assert crc == b["crc"]
        trailer = bytes([b["type"]]) + oracle.mask(crc).to_bytes(4, "little")
        assert trailer.hex() == b["trailer_hex"]


def test_config_blocks(oracle, golden):
    for c in golden["config_blocks"]:
        data = stream_bytes(c["seed"], c["block"] * c["block_bytes"], c["block_bytes"])
        assert oracle.value(data.tobytes()) == c["value"], c


def test_oracle_stream_matches_numpy(oracle):
    for seed, off, n in [(0x5EED0000, 0, 100), (7, 3, 1000), (2**63 + 5, 4095, 333)]:
        assert np.array_equal(oracle.fill_splitmix64(off, n, seed), stream_bytes(seed, off, n))


def test_oracle_batch_drivers(oracle):
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 3000, size=50)
    offs = np.zeros(51, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    data = stream_bytes(99, 0, int(offs[-1]))
    init = rng.integers(0, 2**32, size=50, dtype=np.uint64).astype(np.uint32)
    got = oracle.batch_offsets(data, offs, init, masked=True)
    for i in range(50):
        v = oracle.extend(int(init[i]), data[offs[i]:offs[i + 1]].tobytes())
        assert got[i] == oracle.mask(v)
    fx = oracle.batch_fixed(data, 100, 64, 20)
    assert all(fx[i] == oracle.value(data[i * 100:i * 100 + 64].tobytes()) for i in range(20))


def test_oracle_multithreaded_window_drivers(oracle, golden):
    """The drivers the full-size GPU parity tests use (every config-4 CRC, every
    trailer of a 1M-block SSTable image): a window starting at image byte
    base_off gives the scalar driver's CRCs, and the SSTable driver gives the
    golden trailers of the reference's WriteRawBlock."""
    rng = np.random.default_rng(2)
    lens = rng.integers(0, 5000, size=700)
    lens[::50] = 0
    offs = np.zeros(701, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += 1000
    data = stream_bytes(98, 0, int(offs[-1]) + 7)
    full = oracle.batch_offsets(data, offs)
    for a, b in ((0, 700), (13, 400), (699, 700), (5, 5)):
        base = int(offs[a]) - 3
        win = np.ascontiguousarray(data[base:int(offs[b]) + 2])
        assert np.array_equal(oracle.batch_offsets_mt(win, base, offs[a:b + 1]), full[a:b]), (a, b)
    # SSTable trailers over the golden blocks laid out one after another
    blks = [printable_bytes(x["seed"], x["len"]) for x in golden["sst_blocks"]]
    handles, img, pos = [], [], 77
    for blk in blks:
        handles += [pos, blk.size]
        img.append(blk)
        img.append(np.zeros(5, np.uint8))
        pos += blk.size + 5
    img = np.concatenate([np.zeros(77, np.uint8)] + img)
    types = np.array([x["type"] for x in golden["sst_blocks"]], np.uint8)
    got = oracle.sst_trailers_mt(img[40:], 40, np.array(handles, np.uint64), types)
    assert [oracle.unmask(int(v)) for v in got] == [x["crc"] for x in golden["sst_blocks"]]


def test_sse42_cpu_baseline_matches_the_oracle():
    """bench.py's "not reference" CPU line (oracle/sse42_baseline.c: the x86
    crc32 instruction, three blocks interleaved) computes crc32c::Value
    exactly, for block lengths with and without a word tail and any thread
    count."""
    import ctypes
    import os
    import subprocess
    import numpy as np
    from conftest import Oracle
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(repo, "oracle")], check=True)
    o = Oracle(os.path.join(repo, "oracle", "liboracle_crc32c.so"))
    f = ctypes.CDLL(os.path.join(repo, "oracle", "libsse42_baseline.so")).sse42_batch_fixed_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_int]
    for blen, stride, n, threads in ((4096, 4096, 1001, 3), (4118, 4123, 77, 2), (13, 16, 10, 1), (0, 8, 4, 2)):
        d = np.random.default_rng(blen).integers(0, 256, max(1, n * stride), dtype=np.uint8)
        out = np.empty(n, np.uint32)
        assert f(d.ctypes.data, stride, blen, n, out.ctypes.data, threads) == 0
        assert np.array_equal(out, o.batch_fixed(d, stride, blen, n)), (blen, stride)
