"""Bloom-filter fixture from the REFERENCE's own util/hash.cc, util/bloom.cc
and table/filter_block.cc (compiled in place from /root/reference into
oracle/_ref/libref_bloom.so by `make -C oracle refbloom`).

    python tests/golden/make_bloom_fixture.py

Keys are regenerated from seeds (tests/golden/bloomkeys.py); only the
reference's outputs are stored (tests/golden/bloom_fixture.json):
  * hash: leveldb::Hash of 600 keys (lengths 0..70, all byte values) x 4 seeds;
  * create: CreateFilter bytes (sha256, length, hex when short) for
    bits_per_key x key-count combinations;
  * probe: KeyMayMatch bit strings for members / non-members, for several
    config::bloom_bits_use values, and for hand-made edge filters;
  * blocks: FilterBlockBuilder output for StartBlock/AddKey sequences (db_bench
    shaped, small blocks, gaps with empty filters, no keys, a >8 KiB filter),
    and FilterBlockReader::KeyMayMatch bit strings on the block as built and
    after corruptions of its offset array / trailer.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
from golden.bloomkeys import concat, dbbench_keys, random_keys, take  # noqa: E402

LIB = os.path.join(REPO, "oracle", "_ref", "libref_bloom.so")
vp, sz, u32, u64, i32 = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64,
                         ctypes.c_int)


def load():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "refbloom"], check=True)
    ref = ctypes.CDLL(LIB)
    ref.ref_hash.restype = u32
    ref.ref_hash.argtypes = [vp, sz, u32]
    ref.ref_set_bloom_bits_use.argtypes = [i32]
    ref.ref_create_filter.restype = sz
    ref.ref_create_filter.argtypes = [i32, vp, vp, i32, vp, sz]
    ref.ref_key_may_match.restype = i32
    ref.ref_key_may_match.argtypes = [i32, vp, sz, vp, sz]
    ref.ref_filter_block_build.restype = sz
    ref.ref_filter_block_build.argtypes = [i32, i32, vp, vp, vp, vp, sz, vp, sz]
    ref.ref_filter_block_may_match.restype = i32
    ref.ref_filter_block_may_match.argtypes = [i32, i32, vp, sz, u64, vp, sz]
    return ref


def digest(b):
    b = bytes(b)
    d = {"len": len(b), "sha256": hashlib.sha256(b).hexdigest()}
    if len(b) <= 160:
        d["hex"] = b.hex()
    return d


def buf(a):
    return np.ascontiguousarray(a)


def key_at(keys, i):
    b, o = keys
    return b[int(o[i]):int(o[i + 1])]


# ---- scenario definitions (shared with tests/test_bloom.py through the JSON) ----
CREATE_BPK = [0, 1, 2, 3, 5, 10, 15, 20, 32, 45, 100]
CREATE_N = [0, 1, 2, 3, 7, 33, 100, 700]
PROBE_BBU = [15, 0, 3, 40]


def block_scenarios():
    """(name, strip, bits_per_key, keyspec, block_start, block_first)."""
    out = []
    # db_bench shaped: 60 data blocks of ~4123 B with 33 internal keys each
    rng = np.random.default_rng(0xB10C)
    starts, pos = [], 0
    for _ in range(60):
        starts.append(pos)
        pos += 4118 + int(rng.integers(0, 4)) + 5
    starts.append(pos)  # Finish()'s Flush: StartBlock after the last block
    first = [33 * i for i in range(61)] + [33 * 60]
    out.append(("dbbench", 8, 20, {"kind": "dbbench", "first": 1000, "n": 33 * 60},
                starts, first))
    # small blocks (several per 2 KiB filter), user keys with all byte values
    starts, first, pos, k = [], [0], 0, 0
    for i in range(120):
        starts.append(pos)
        pos += int(rng.integers(200, 1500))
        k += int(rng.integers(1, 9))
        first.append(k)
    out.append(("small_blocks", 0, 10, {"kind": "random", "seed": 0xB2, "n": k, "lo": 1, "hi": 40},
                starts, first))
    # gaps: empty filters between blocks, a block without keys, a trailing
    # StartBlock far past the last filter
    starts = [0, 100, 9000, 9001, 30000, 30500, 31000, 70000]
    first = [0, 5, 9, 9, 20, 24, 31, 31, 31]
    out.append(("gaps", 8, 15, {"kind": "dbbench", "first": 77, "n": 31}, starts, first))
    # no keys at all
    out.append(("no_keys", 0, 20, {"kind": "random", "seed": 3, "n": 0, "lo": 0, "hi": 0},
                [0, 4096, 8192], [0, 0, 0, 0]))
    out.append(("only_start", 0, 20, {"kind": "random", "seed": 3, "n": 0, "lo": 0, "hi": 0},
                [0], [0, 0]))
    # one big filter (> the GPU's per-wave LDS window), then a small one
    out.append(("big_filter", 0, 20, {"kind": "random", "seed": 0xB16, "n": 5100, "lo": 0,
                                      "hi": 24},
                [0, 1 << 20], [0, 5000, 5100]))
    # many empty filters then keys (index > 255 filters)
    out.append(("late_keys", 8, 10, {"kind": "dbbench", "first": 5, "n": 40},
                [0, 600000, 600100], [0, 0, 30, 40]))
    return out


def make_keys(spec):
    if spec["kind"] == "dbbench":
        return dbbench_keys(spec["first"], spec["n"])
    return random_keys(spec["seed"], spec["n"], spec["lo"], spec["hi"])


def corruptions(block):
    """(name, ops) applied to a built filter block (little-endian fields)."""
    n = len(block)
    if n < 5:
        return []
    last_word = int.from_bytes(bytes(block[n - 5:n - 1]), "little")
    num = (n - 5 - last_word) // 4
    ops = [("as_built", []),
           ("truncated_4", [["truncate", 4]]),
           ("last_word_past_end", [["set", n - 5, (n - 4).to_bytes(4, "little").hex()]]),
           ("base_lg_0", [["set", n - 1, "00"]]),
           ("base_lg_12", [["set", n - 1, "0c"]]),
           ("base_lg_negative", [["set", n - 1, "ff"]])]
    if num >= 2:
        o1 = last_word + 4
        ops.append(("start_after_limit", [["set", o1, (0xFFFFFF).to_bytes(4, "little").hex()]]))
        ops.append(("limit_past_array", [["set", last_word + 4 * min(num, 2),
                                          (last_word + 1).to_bytes(4, "little").hex()]]))
        ops.append(("all_empty", [["set", last_word + 4 * i, "00000000"] for i in range(num)]))
    return ops


def apply(img, ops):
    img = bytearray(img)
    for op in ops:
        if op[0] == "set":
            b = bytes.fromhex(op[2])
            img[op[1]:op[1] + len(b)] = b
        elif op[0] == "truncate":
            img = img[:op[1]]
    return bytes(img)


def main():
    ref = load()
    fx = {"source": "lsbm util/hash.cc, util/bloom.cc, table/filter_block.cc built from "
                    "/root/reference (oracle/Makefile refbloom); tests/golden/make_bloom_fixture.py"}
    # ---- hash
    hk = random_keys(0xB100, 600, 0, 70)
    fx["hash"] = {"keys": {"seed": 0xB100, "n": 600, "lo": 0, "hi": 70}, "values": {}}
    for seed in [0xBC9F1D34, 0, 0xFFFFFFFF, 0x12345678]:
        fx["hash"]["values"][str(seed)] = [
            int(ref.ref_hash(buf(key_at(hk, i)).ctypes.data, int(hk[1][i + 1] - hk[1][i]), seed))
            for i in range(600)]
    # ---- create
    fx["create"] = []
    for bpk in CREATE_BPK:
        for n in CREATE_N:
            seed = 0xC000 + 97 * bpk + n
            b, o = random_keys(seed, n, 0, 40)
            out = ctypes.create_string_buffer(1 << 20)
            k = ref.ref_create_filter(bpk, buf(b).ctypes.data, buf(o).ctypes.data, n, out, 1 << 20)
            fx["create"].append({"bits_per_key": bpk, "n": n, "seed": seed, "lo": 0, "hi": 40,
                                 **digest(out.raw[:k])})
    # ---- probe
    fx["probe"] = []
    for bpk in [10, 20]:
        members = random_keys(0xD000 + bpk, 200, 1, 30, printable=True)
        others = random_keys(0xD100 + bpk, 300, 1, 30, printable=True)
        out = ctypes.create_string_buffer(1 << 16)
        k = ref.ref_create_filter(bpk, buf(members[0]).ctypes.data, buf(members[1]).ctypes.data,
                                  200, out, 1 << 16)
        filt = out.raw[:k]
        probes = concat(members, others)
        for bbu in PROBE_BBU:
            ref.ref_set_bloom_bits_use(bbu)
            bits = "".join(str(ref.ref_key_may_match(bpk, buf(key_at(probes, i)).ctypes.data,
                                                     int(probes[1][i + 1] - probes[1][i]),
                                                     filt, len(filt)))
                           for i in range(500))
            fx["probe"].append({"bits_per_key": bpk, "bloom_bits_use": bbu,
                                "members": {"seed": 0xD000 + bpk, "n": 200},
                                "others": {"seed": 0xD100 + bpk, "n": 300},
                                "filter": digest(filt), "may": bits})
    ref.ref_set_bloom_bits_use(15)
    # hand-made filters: empty, 1 byte, k byte 31 / 0x85 (negative) / 0 / 2
    edge_keys = random_keys(0xE0, 64, 0, 20)
    fx["probe_edge"] = []
    for name, hexf in [("len0", ""), ("len1", "05"), ("k31", "ff" * 8 + "1f"),
                       ("k_negative", "5a" * 16 + "85"), ("k0", "00" * 8 + "00"),
                       ("k2", "a5c3" * 6 + "02"), ("k14_over_use", "ff" * 20 + "0e")]:
        f = bytes.fromhex(hexf)
        for bpk in [10, 20]:
            bits = "".join(str(ref.ref_key_may_match(bpk, buf(key_at(edge_keys, i)).ctypes.data,
                                                     int(edge_keys[1][i + 1] - edge_keys[1][i]),
                                                     f, len(f)))
                           for i in range(64))
            fx["probe_edge"].append({"name": name, "filter_hex": hexf, "bits_per_key": bpk,
                                     "keys": {"seed": 0xE0, "n": 64, "lo": 0, "hi": 20},
                                     "may": bits})
    # ---- filter blocks
    fx["blocks"] = []
    for name, strip, bpk, spec, starts, first in block_scenarios():
        keys = make_keys(spec)
        st = np.array(starts, dtype=np.uint64)
        fi = np.array(first, dtype=np.uint64)
        nb = len(starts)
        assert fi.size >= nb + 1
        out = ctypes.create_string_buffer(1 << 22)
        k = ref.ref_filter_block_build(bpk, strip, buf(keys[0]).ctypes.data,
                                       buf(keys[1]).ctypes.data, st.ctypes.data, fi.ctypes.data,
                                       nb, out, 1 << 22)
        block = out.raw[:k]
        # lookups: every member key at its own block's offset, non-members at
        # member offsets, and offsets past the last filter
        nk = int(spec["n"])
        q_keys, q_off = [], []
        blk_of = np.searchsorted(fi[1:nb + 1], np.arange(nk), side="right")
        for i in range(nk):
            q_keys.append(key_at(keys, i))
            q_off.append(starts[int(blk_of[i])])
        strip_pad = bytes(strip)
        others = random_keys(0xF000 + len(fx["blocks"]), 64, 1, 30)
        for i in range(64):
            q_keys.append(np.frombuffer(bytes(key_at(others, i)) + strip_pad, np.uint8))
            q_off.append(starts[i % nb])
        for off in [starts[-1] + 4096, 1 << 40, 2047, 2048]:
            q_keys.append(key_at(keys, 0) if nk else np.frombuffer(b"x" * (strip + 1), np.uint8))
            q_off.append(off)
        scen = []
        for cname, ops in corruptions(block):
            img = apply(block, ops)
            bits = "".join(str(ref.ref_filter_block_may_match(
                bpk, strip, img, len(img), int(q_off[j]), buf(q_keys[j]).ctypes.data,
                len(q_keys[j]))) for j in range(len(q_keys)))
            scen.append({"name": cname, "ops": ops, "may": bits})
        fx["blocks"].append({"name": name, "strip": strip, "bits_per_key": bpk, "keys": spec,
                             "block_start": starts, "block_first": first,
                             "block": digest(block),
                             "queries": {"others_seed": 0xF000 + len(fx["blocks"]),
                                         "offsets": [int(x) for x in q_off]},
                             "lookups": scen})
    with open(os.path.join(HERE, "bloom_fixture.json"), "w") as f:
        json.dump(fx, f, indent=0)
    print(f"hash {len(fx['hash']['values'])}x600, create {len(fx['create'])}, "
          f"probe {len(fx['probe'])}+{len(fx['probe_edge'])}, blocks {len(fx['blocks'])} "
          f"({sum(len(b['lookups']) for b in fx['blocks'])} lookup scenarios)")


if __name__ == "__main__":
    sys.exit(main())
