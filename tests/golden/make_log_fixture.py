"""WAL fixture written and read by the REFERENCE's own log::Writer / log::Reader
(common/log_writer.cc, common/log_reader.cc, compiled in place from
/root/reference into oracle/_ref/libref_log.so by `make -C oracle reflog`).

    python tests/golden/make_log_fixture.py

Records: a seeded list of lengths chosen to hit every framing case of
log::Writer::AddRecord (common/log_writer.cc:27-73): empty records, FULL
records, block trailers of 1..6 zero bytes, a record ending exactly at a block
boundary, FIRST/LAST and FIRST/MIDDLE/LAST fragments, db_bench-sized records.
Payload bytes: printable_bytes(seed, total) (tests/golden/splitmix.py).

Stored (tests/golden/log_fixture.json), no image bytes:
  * lens / seed of the records;
  * the reference writer's image as length + crc32c + every header's 4 CRC
    bytes (enough to rebuild it exactly from a layout with blank CRCs);
  * corruption scenarios (byte xors / sets / zeroed ranges / truncation applied to that
    image) with the reference reader's exact output for each: every
    ReadRecord result (length, crc32c, LastRecordOffset) and every
    Reporter::Corruption call (bytes, status), in order.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from splitmix import printable_bytes  # noqa: E402

LIB = os.path.join(REPO, "oracle", "_ref", "libref_log.so")
BLOCK, HEADER = 32768, 7  # common/log_format.h:27-30
SEED = 0x106F17E


def frame_offsets(lens):
    """Header offsets of every physical record (log::Writer framing)."""
    pos, bo, heads, types = 0, 0, [], []
    for n in lens:
        left, first = n, True
        while True:
            if BLOCK - bo < HEADER:
                pos += BLOCK - bo
                bo = 0
            frag = min(left, BLOCK - bo - HEADER)
            last = frag == left
            heads.append(pos)
            types.append((1 if last else 2) if first else (4 if last else 3))
            pos += HEADER + frag
            bo += HEADER + frag
            left -= frag
            first = False
            if left == 0:
                break
    return heads, types, bo


def record_lengths():
    rng = np.random.default_rng(SEED)
    lens = [0, 1, 6, 7, 100, 0]
    for k in range(1, 7):  # a block trailer of exactly k zero bytes
        while frame_offsets(lens)[2] < 30000:
            lens.append(int(rng.integers(0, 2541)))  # db_bench-like, mean ~1270
        bo = frame_offsets(lens)[2]
        lens.append(BLOCK - k - HEADER - bo)
        lens.append(int(rng.integers(1, 200)))  # starts the next block after the pad
    # a record that ends exactly at a block boundary (leftover 0, no pad)
    while frame_offsets(lens)[2] < 30000:
        lens.append(int(rng.integers(0, 2541)))
    lens.append(BLOCK - HEADER - frame_offsets(lens)[2])
    lens += [BLOCK - HEADER, BLOCK - HEADER + 1, 70000, 0, 3]  # FULL at 0, FIRST/LAST, F/M/M/L
    lens += [int(x) for x in rng.integers(0, 4000, size=40)]
    return lens


def main():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "reflog"], check=True)
    ref = ctypes.CDLL(LIB)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    ref.ref_log_write.restype = sz
    ref.ref_log_write.argtypes = [vp, vp, sz, vp, sz]
    ref.ref_log_read.restype = sz
    ref.ref_log_read.argtypes = [vp, sz, vp, sz]
    ref.ref_log_read_from.restype = sz
    ref.ref_log_read_from.argtypes = [vp, sz, ctypes.c_uint64, vp, sz]
    ref.ref_log_value.restype = ctypes.c_uint32
    ref.ref_log_value.argtypes = [vp, sz]

    lens = record_lengths()
    payload = printable_bytes(SEED, int(sum(lens)))
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    cap = int(sum(lens)) + 64 * len(lens) + (1 << 20)
    out = ctypes.create_string_buffer(cap)
    n = ref.ref_log_write(payload.ctypes.data, offs.ctypes.data, len(lens), out, cap)
    image = np.frombuffer(out.raw[:n], dtype=np.uint8).copy()
    heads, types, _ = frame_offsets(lens)
    assert heads[-1] < n and all(image[h + 6] == t for h, t in zip(heads, types))

    def value(buf):
        b = np.ascontiguousarray(buf, dtype=np.uint8)
        return int(ref.ref_log_value(b.ctypes.data, b.size))

    def read(img):
        b = np.ascontiguousarray(img, dtype=np.uint8)
        o = ctypes.create_string_buffer(1 << 22)
        k = ref.ref_log_read(b.ctypes.data, b.size, o, 1 << 22)
        return o.raw[:k].decode()

    def read_from(img, off):
        b = np.ascontiguousarray(img, dtype=np.uint8)
        o = ctypes.create_string_buffer(1 << 22)
        k = ref.ref_log_read_from(b.ctypes.data, b.size, off, o, 1 << 22)
        return o.raw[:k].decode()

    def apply(img, ops):
        img = img.copy()
        for op in ops:
            if op[0] == "xor":
                img[op[1]] ^= op[2]
            elif op[0] == "set":
                img[op[1]:op[1] + len(op[2]) // 2] = np.frombuffer(bytes.fromhex(op[2]), np.uint8)
            elif op[0] == "zero":
                img[op[1]:op[1] + op[2]] = 0
            elif op[0] == "truncate":
                img = img[:op[1]]
        return img

    def recrc(img, h):
        """'set' op rewriting header h's CRC for its current type/length."""
        length = int(img[h + 4]) | int(img[h + 5]) << 8
        c = value(img[h + 6:h + 7 + length])
        m = (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF  # util/crc32c.h Mask
        return ["set", h, m.to_bytes(4, "little").hex()]

    by_type = {t: [h for h, tt in zip(heads, types) if tt == t] for t in (1, 2, 3, 4)}
    full0 = by_type[1][3]
    first, middle = by_type[2][0], by_type[3][0]
    first3 = [h for h, t, t2 in zip(heads, types, types[1:]) if t == 2 and t2 == 3][0]
    lastblock = (n - 1) // BLOCK * BLOCK
    tail_heads = [h for h in heads if h >= lastblock]
    rng = np.random.default_rng(SEED + 1)
    scen = [
        ("clean", []),
        ("payload_flip_full", [["xor", full0 + HEADER + 3, 0x10]]),
        ("crc_field_flip", [["xor", by_type[1][10] + 1, 0x01]]),
        ("type_byte_flip", [["xor", by_type[1][11] + 6, 0x02]]),
        ("payload_flip_first", [["xor", first + HEADER + 5, 0x40]]),
        ("payload_flip_middle", [["xor", middle + HEADER + 100, 0x04]]),
        ("payload_flip_first_of_three", [["xor", first3 + HEADER + 9, 0x08]]),
        ("length_past_block", [["set", by_type[1][12] + 4, "ff7f"]]),
        ("truncate_mid_payload", [["truncate", tail_heads[-1] + HEADER + 1]]),
        ("truncate_mid_header", [["truncate", tail_heads[-1] + 3]]),
        ("truncate_in_fragmented", [["truncate", by_type[4][-1] + 2]]),
        ("zero_block", [["zero", BLOCK * 2, BLOCK]]),
        ("zero_block_in_fragmented", [["zero", (middle // BLOCK) * BLOCK, BLOCK]]),
    ]
    # type rewrites with a valid CRC: unknown types, the 5 / 6 aliases of
    # kEof / kBadRecord, a sign-extended type, FIRST turned into FULL
    for name, h, t in [("type_9", by_type[1][13], 9), ("type_5_reads_as_eof", by_type[1][14], 5),
                       ("type_6_reads_as_bad", by_type[1][15], 6),
                       ("type_0x85_sign_extended", by_type[1][16], 0x85),
                       ("first_as_full", first, 1), ("last_as_middle", by_type[4][0], 3),
                       ("middle_as_full", middle, 1),
                       ("zero_type_nonempty", by_type[1][17], 0)]:
        img = apply(image, [["set", h + 6, "%02x" % t]])
        scen.append((name, [["set", h + 6, "%02x" % t], recrc(img, h)]))
    # a zero-length zero-type header mid-block: the rest of the block is skipped silently
    h = by_type[1][18]
    scen.append(("zero_header_skip", [["set", h, "00" * HEADER]]))
    for k in range(3):
        flips = [["xor", int(o), int(rng.integers(1, 256))]
                 for o in rng.choice(n, size=12 * (k + 1), replace=False)]
        scen.append((f"random_flips_{k}", flips))

    scenarios = []
    for name, ops in scen:
        scenarios.append({"name": name, "ops": ops, "events": read(apply(image, ops))})
    # log::Reader with initial_offset != 0 (SkipToInitialBlock, the skip of
    # physical records that start before the offset, unreported drops before
    # it: common/log_reader.cc:35-57, 171-176, 247-251)
    last = by_type[4][0]
    offs_cases = [
        ("at_zero", [], 0), ("one", [], 1), ("at_full_header", [], by_type[1][5]),
        ("inside_full", [], by_type[1][5] + 9), ("at_first", [], first),
        ("inside_first", [], first + 30), ("inside_middle", [], middle + 500),
        ("inside_last", [], last + 11), ("block_1", [], BLOCK), ("block_1_minus_6", [], BLOCK - 6),
        ("block_1_minus_5", [], BLOCK - 5), ("block_1_minus_1", [], BLOCK - 1),
        ("block_2_plus_100", [], 2 * BLOCK + 100), ("near_end", [], n - 3), ("at_end", [], n),
        ("past_end", [], n + 5000), ("far_past_end", [], n + 10 * BLOCK),
        ("flip_before_offset_block", [["xor", full0 + HEADER + 3, 0x10]], BLOCK * (full0 // BLOCK + 1)),
        ("flip_before_offset_same_block", [["xor", by_type[1][6] + HEADER + 1, 0x10]],
         by_type[1][6] + 40),
        ("flip_after_offset", [["xor", by_type[1][20] + HEADER + 2, 0x01]], by_type[1][19]),
        ("truncated_after_offset", [["truncate", tail_heads[-1] + 3]], tail_heads[0]),
    ]
    offset_scenarios = []
    for name, ops, off in offs_cases:
        offset_scenarios.append({"name": name, "ops": ops, "initial_offset": int(off),
                                 "events": read_from(apply(image, ops), int(off))})
    assert offset_scenarios[0]["events"] == scenarios[0]["events"]
    fixture = {
        "source": "lsbm common/log_writer.cc + common/log_reader.cc built from /root/reference "
                  "(oracle/Makefile reflog); tests/golden/make_log_fixture.py",
        "seed": SEED, "lens": lens,
        "image": {"bytes": int(n), "crc32c": value(image),
                  "header_crcs": [image[h:h + 4].tobytes().hex() for h in heads]},
        "scenarios": scenarios,
        "offset_scenarios": offset_scenarios,
    }
    with open(os.path.join(HERE, "log_fixture.json"), "w") as f:
        json.dump(fixture, f, indent=0)
    kinds = sorted({line.split(" ", 2)[2] if line.startswith("D") else "R"
                    for s in scenarios for line in s["events"].splitlines()})
    print(f"{len(lens)} records, {len(heads)} physical, image {n} B, "
          f"{len(scenarios)} scenarios, {len(offset_scenarios)} initial-offset scenarios; "
          f"event kinds: {kinds}")


if __name__ == "__main__":
    sys.exit(main())
