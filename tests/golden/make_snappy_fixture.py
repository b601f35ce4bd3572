"""Regenerate tests/golden/snappy_fixture.json from the libsnappy inside the
image's pyarrow (pyarrow.Codec("snappy") = snappy::RawCompress /
snappy::RawUncompress, the functions port/port_posix.h:119-150 of the
reference calls).  libsnappy itself is not part of /root/reference; this pins
oracle/snappy_oracle.c to a real build of it.

    python tests/golden/make_snappy_fixture.py

Records, per case: the block spec (kind, length, seed, see snappy_inputs.py),
the compressed length and sha256 of RawCompress's output, the first bytes of
it, and the 12.5% rule's choice (table/table_builder.cc:187-188).  Corruption
cases apply a mutation to a compressed block and record whether RawUncompress
accepts it and the sha256 of what it produced.
"""
import hashlib
import json
import os
import sys

import pyarrow as pa

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from snappy_inputs import KINDS, block, mutations, varint32  # noqa: E402

CODEC = pa.Codec("snappy")


def compress(d):
    return CODEC.compress(d, asbytes=True)


def uncompress(c):
    """(ok, output) of snappy::RawUncompress, as Arrow's SnappyCodec calls it."""
    ulen = 0
    for i, b in enumerate(c[:5]):
        if i == 4 and b >= 16:
            ulen = 0
            break
        ulen |= (b & 127) << (7 * i)
        if b < 128:
            break
    else:
        ulen = 0
    try:
        # decompressed_size must be the exact length: Arrow returns a buffer of that size
        return True, CODEC.decompress(c, decompressed_size=ulen, asbytes=True)
    except OSError:
        return False, b""


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    lengths = [0, 1, 2, 3, 4, 14, 15, 16, 17, 31, 32, 33, 60, 61, 64, 65, 100, 255, 256, 257,
               1000, 2047, 2048, 2049, 4095, 4096, 4097, 4117, 4118, 4122, 8192, 16383, 16384,
               16385, 32768, 32769, 65535, 65536, 65537, 70000, 131072, 200001]
    cases = []
    seed = 1000
    for kind in KINDS:
        for n in lengths:
            seed += 1
            d = block(kind, n, seed)
            c = compress(d)
            assert uncompress(c) == (True, d)
            cases.append({"kind": kind, "n": n, "seed": seed, "clen": len(c), "csha": sha(c),
                          "head": c[:24].hex(),
                          "store_compressed": len(c) < n - n // 8})
    corrupt = []
    for i, cs in enumerate(cases):
        if cs["n"] not in (17, 100, 4118, 65537) or cs["kind"] in ("zeros",):
            continue
        c = compress(block(cs["kind"], cs["n"], cs["seed"]))
        for name, m in mutations(c, 7000 + i):
            ok, out = uncompress(m)
            corrupt.append({"case": i, "mutation": name, "ok": ok,
                            "out_sha": sha(out) if ok else None, "out_len": len(out)})
    crafted = {
        "empty": b"",
        "zero_len": b"\x00",
        "zero_len_trailing": b"\x00\x00",
        "one_literal": b"\x01\x00a",
        "literal_ext1": varint32(61) + bytes([60 << 2, 60]) + b"x" * 61,
        "literal_ext2": varint32(300) + bytes([61 << 2]) + (299).to_bytes(2, "little") + b"y" * 300,
        "literal_ext3": varint32(70000) + bytes([62 << 2]) + (69999).to_bytes(3, "little") + b"z" * 70000,
        "literal_ext4": varint32(5) + bytes([63 << 2]) + (4).to_bytes(4, "little") + b"w" * 5,
        "literal_short_input": varint32(10) + bytes([9 << 2]) + b"abc",
        "literal_over_ulen": varint32(2) + bytes([3 << 2]) + b"abcd",
        "copy1_rle": varint32(12) + b"\x00a" + bytes([1 | ((19 - 4) & 7) << 2]) + b"\x01",
        "copy1_ok": varint32(9) + b"\x00a" + bytes([1 | (4 << 2)]) + b"\x01",
        "copy1_offset0": varint32(9) + b"\x00a" + bytes([1 | (4 << 2)]) + b"\x00",
        "copy1_offset_past": varint32(9) + b"\x00a" + bytes([1 | (4 << 2)]) + b"\x02",
        "copy2_ok": varint32(65) + b"\x00a" + bytes([2 | (63 << 2)]) + b"\x01\x00",
        "copy2_truncated": varint32(65) + b"\x00a" + bytes([2 | (63 << 2)]) + b"\x01",
        "copy4_ok": varint32(33) + b"\x00a" + bytes([3 | (31 << 2)]) + b"\x01\x00\x00\x00",
        "copy4_big_offset": varint32(33) + b"\x00a" + bytes([3 | (31 << 2)]) + b"\x00\x00\x01\x00",
        "copy_over_ulen": varint32(8) + b"\x00a" + bytes([1 | (4 << 2)]) + b"\x01",
        "short_output": varint32(9) + b"\x00a",
        "varint_5byte_ok": bytes([0x80, 0x80, 0x80, 0x80, 0x00]),
        "varint_5th_ge16": bytes([0x80, 0x80, 0x80, 0x80, 0x10]),
        "varint_unterminated": bytes([0x80, 0x80]),
        "varint_6byte": bytes([0x80, 0x80, 0x80, 0x80, 0x80, 0x00]),
        "tag_only": varint32(1) + b"\x00",
    }
    crafted_rec = []
    for name, m in crafted.items():
        ok, out = uncompress(m)
        crafted_rec.append({"name": name, "hex": m.hex() if len(m) < 512 else None,
                            "ok": ok, "out_len": len(out), "out_sha": sha(out) if ok else None})
    # the long literal case is stored by construction, not as hex
    fx = {"source": "libsnappy inside pyarrow %s (snappy::RawCompress / RawUncompress)" % pa.__version__,
          "cases": cases, "corrupt": corrupt, "crafted": crafted_rec}
    with open(os.path.join(here, "snappy_fixture.json"), "w") as f:
        json.dump(fx, f, indent=0)
    print(len(cases), "cases,", len(corrupt), "corruptions,", len(crafted_rec), "crafted")


if __name__ == "__main__":
    main()
