"""Deterministic block contents for the snappy fixtures and tests.

`block(kind, n, seed)` builds n bytes of one of several shapes, from numpy's
PCG64 (stable across numpy releases for `integers`): uniform random bytes
(incompressible), 2-bit symbols, printable text, leveldb-like key/value records
(`table/block_builder.cc` prefix-compressed entries look like this: short
varint headers, shared key prefixes, repeated values), zeros, and a short
random period (long overlapping copies).  The generator is shared by the
fixture script and the tests so that only specs, lengths and digests are
committed.
"""
import numpy as np

KINDS = ("random", "bits2", "printable", "records", "zeros", "period")



def block(kind, n, seed):
    rng = np.random.default_rng(seed)
    if n == 0:
        return b""
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "bits2":
        return rng.integers(0, 4, n, dtype=np.uint8).tobytes()
    if kind == "printable":
        return rng.integers(32, 127, n, dtype=np.uint8).tobytes()
    if kind == "records":
        out, k = [], int(rng.integers(0, 10**6))
        size = 0
        while size < n:
            k += int(rng.integers(1, 50))
            vlen = int(rng.integers(0, 120))
            val = bytes(rng.integers(97, 101, vlen, dtype=np.uint8)) if vlen else b""
            rec = bytes([int(rng.integers(0, 16)), 16, vlen & 127]) + b"user%012d" % k + val
            out.append(rec)
            size += len(rec)
        return b"".join(out)[:n]
    if kind == "zeros":
        return bytes(n)
    if kind == "period":
        p = int(rng.integers(1, 40))
        unit = rng.integers(0, 256, p, dtype=np.uint8).tobytes()
        return (unit * (n // p + 1))[:n]
    raise ValueError(kind)


def dbbench_block(seed, first_key, block_size=4096, value_size=100, ratio=0.5, seq0=1):
    """A data block as db_bench's fill workload writes it:
    BlockBuilder layout (table/block_builder.cc: restart every 16 entries,
    shared / non-shared / value-length varints, key delta, value; restart
    array and count at the end) over internal keys "user%019d" + 8-byte
    (seq << 8 | 1), with 100-byte values that compress to ~50%
    (util/testutil.cc CompressibleString: 50 random printable bytes, repeated).
    Returns (block bytes, next key)."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    restarts, last, k, count = [], b"", first_key, 0
    while len(out) + 4 * (len(restarts) + 1) < block_size:
        key = b"user%019d" % k + ((seq0 + k) << 8 | 1).to_bytes(8, "little")
        raw = bytes(rng.integers(32, 127, int(value_size * ratio), dtype=np.uint8))
        val = (raw * (value_size // len(raw) + 1))[:value_size]
        if count % 16 == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(last), len(key)) and last[shared] == key[shared]:
                shared += 1
        out += varint32(shared) + varint32(len(key) - shared) + varint32(len(val))
        out += key[shared:] + val
        last, k, count = key, k + 1, count + 1
    for r in restarts:
        out += r.to_bytes(4, "little")
    out += len(restarts).to_bytes(4, "little")
    return bytes(out), k


def varint32(v):
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def mutations(c, seed):
    """Deterministic corruptions of compressed block c: (name, bytes)."""
    rng = np.random.default_rng(seed)
    out = [("truncate_1", c[:-1]), ("truncate_half", c[: len(c) // 2]), ("append_zero", c + b"\0"),
           ("append_literal", c + b"\x00A")]
    for j in range(4):
        p = int(rng.integers(0, len(c)))
        v = int(rng.integers(0, 256))
        out.append(("set_%d_%d" % (p, v), c[:p] + bytes([v]) + c[p + 1:]))
    return out
