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


def varint32(v):
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)
