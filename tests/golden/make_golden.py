"""Generate tests/golden/crc32c_golden.json from the REFERENCE's own CRC-32C.

Run in the build container only (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

The expected values come from oracle/_ref/libref_crc32c.so, i.e. lsbm's
util/crc32c.cc (Extend, :286-329) and util/crc32c.h (Value/Mask/Unmask,
:20-40) compiled unmodified from /root/reference.  Inputs are stored as
generator specs (seeded splitmix64 streams, tests/golden/splitmix.py) so the
fixture stays small; the reference itself never leaves this container.
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from golden.splitmix import printable_bytes, stream_bytes  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
REF = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so"))
REF.ref_extend.restype = ctypes.c_uint32
REF.ref_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
REF.ref_mask.restype = ctypes.c_uint32
REF.ref_mask.argtypes = [ctypes.c_uint32]
REF.ref_unmask.restype = ctypes.c_uint32
REF.ref_unmask.argtypes = [ctypes.c_uint32]


def ref_extend(init, data, align=0):
    """Call the reference Extend with the data placed at byte offset `align`
    of a 64-byte aligned buffer (the reference byte-steps to 4-byte alignment,
    util/crc32c.cc:304-313; the result must not depend on it)."""
    data = bytes(data)
    buf = ctypes.create_string_buffer(len(data) + 128)
    base = (ctypes.addressof(buf) + 63) & ~63
    ctypes.memmove(base + align, data, len(data))
    return REF.ref_extend(init & 0xFFFFFFFF, base + align, len(data))


def main():
    out = {"source": "reference util/crc32c.cc compiled from /root/reference "
                     "(oracle/Makefile target ref)",
           "stream": "splitmix64, tests/golden/splitmix.py"}

    # 1. known-answer tests (RFC 3720 B.4 iSCSI vectors + strings).
    kat = [
        ("zeros32", bytes(32)),
        ("ones32", b"\xff" * 32),
        ("inc32", bytes(range(32))),
        ("dec32", bytes(range(31, -1, -1))),
        ("123456789", b"123456789"),
        ("empty", b""),
        ("a", b"a"),
        ("hello world", b"hello world"),
        ("foo", b"foo"),
    ]
    out["kat"] = [{"name": n, "hex": d.hex(), "value": ref_extend(0, d),
                   "mask": REF.ref_mask(ref_extend(0, d))} for n, d in kat]
    hv = ref_extend(0, b"hello ")
    out["extend_chain"] = {"a": "hello ", "b": "world", "value_a": hv,
                           "extend": ref_extend(hv, b"world")}
    foo = ref_extend(0, b"foo")
    out["mask_chain"] = {"crc": foo, "mask": REF.ref_mask(foo),
                         "mask2": REF.ref_mask(REF.ref_mask(foo))}

    # 2. seeded random (len, align, init, seed) cases.
    rng = np.random.default_rng(20261015)
    fixed_lens = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64,
                  65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024,
                  1025, 4095, 4096, 4097, 4117, 4118, 4119, 4120, 4121, 4122,
                  8191, 8192, 65535, 65536]
    cases = []
    for k in range(4096):
        if k < len(fixed_lens) * 4:
            n = fixed_lens[k // 4]
        elif k % 4 == 0:
            n = int(rng.integers(0, 70001))
        else:
            n = int(rng.integers(0, 4200))
        align = int(rng.integers(0, 16))
        init = 0 if k % 3 == 0 else int(rng.integers(0, 2**32))
        seed = int(rng.integers(0, 2**63))
        v = ref_extend(init, stream_bytes(seed, 0, n).tobytes(), align)
        cases.append({"len": n, "align": align, "init": init, "seed": seed,
                      "value": v, "mask": REF.ref_mask(v)})
    out["random"] = cases

    # 3. SSTable block trailers, table/table_builder.cc:237-255:
    #    crc = Value(block, n); crc = Extend(crc, &type, 1); trailer =
    #    [type][EncodeFixed32(Mask(crc))].  db_bench-sized printable blocks.
    blocks = []
    for k in range(64):
        n = 4117 + (k % 6)
        seed = 0xB10C0000 + k
        typ = 0 if k % 8 else 1
        blk = printable_bytes(seed, n).tobytes()
        crc = ref_extend(ref_extend(0, blk), bytes([typ]))
        assert crc == ref_extend(0, blk + bytes([typ]))
        m = REF.ref_mask(crc)
        blocks.append({"len": n, "seed": seed, "type": typ, "crc": crc,
                       "trailer_hex": (bytes([typ]) + m.to_bytes(4, "little")).hex()})
    out["sst_blocks"] = blocks

    # 4. benchmark-config spot checks: first blocks of each config buffer.
    cfg = []
    for name, seed, bsz in [("cfg2_4k", 0x5EED0000, 4096), ("cfg3_64k", 0x5EED0001, 65536)]:
        for b in [0, 1, 2, 3, 1000, 65537]:
            data = stream_bytes(seed, b * bsz, bsz).tobytes()
            cfg.append({"config": name, "seed": seed, "block": b, "block_bytes": bsz,
                        "value": ref_extend(0, data)})
    # config 5 (80M x 4 KiB over 8 shards of 10M, the same stream as config 2):
    # the blocks either side of every shard boundary, and the last block
    for b in [10_000_000 * r + d for r in range(1, 8) for d in (-1, 0)] + [79_999_999]:
        data = stream_bytes(0x5EED0000, b * 4096, 4096).tobytes()
        cfg.append({"config": "cfg5_shards", "seed": 0x5EED0000, "block": b, "block_bytes": 4096,
                    "value": ref_extend(0, data)})
    out["config_blocks"] = cfg

    path = os.path.join(HERE, "crc32c_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
