"""Seeded key sets for the bloom-filter fixtures and tests.

Keys are stored flat: one uint8 buffer plus uint64 offsets (key i =
buf[offs[i], offs[i+1])), the layout every bloom entry point takes.
"""
import numpy as np

from .splitmix import splitmix64, stream_bytes


def _lengths(seed, n, lo, hi):
    with np.errstate(over="ignore"):
        r = splitmix64(np.uint64(seed) + np.arange(n, dtype=np.uint64))
    return (lo + (r % np.uint64(hi - lo + 1)).astype(np.int64)).astype(np.int64)


def random_keys(seed, n, lo=0, hi=40, printable=False):
    """n keys of lengths U[lo, hi]; bytes from the splitmix stream `seed`
    (all 256 values, so the signed-char tail of util/hash.cc:35-47 is hit),
    or db_bench-like printable bytes."""
    lens = _lengths(seed ^ 0x5A5A, n, lo, hi)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    buf = stream_bytes(seed, 0, int(offs[-1]))
    if printable:
        buf = (np.uint8(32) + buf % np.uint8(95)).astype(np.uint8)
    return buf, offs


def dbbench_keys(first, n, seq0=1, internal=True):
    """db_bench keys "user%019d" (lsbm/db_bench.cc:1415) for key numbers
    first..first+n-1; internal keys append the 8-byte little-endian
    (sequence << 8 | kTypeValue) suffix (common/dbformat.h)."""
    klen = 23 + (8 if internal else 0)
    out = np.empty((n, klen), dtype=np.uint8)
    nums = np.arange(first, first + n, dtype=np.int64)
    out[:, :4] = np.frombuffer(b"user", dtype=np.uint8)
    for p in range(19):
        out[:, 4 + p] = (48 + (nums // 10 ** (18 - p)) % 10).astype(np.uint8)
    if internal:
        tag = (np.arange(seq0, seq0 + n, dtype=np.uint64) << np.uint64(8)) | np.uint64(1)
        out[:, 23:] = tag.astype("<u8").view(np.uint8).reshape(n, 8)
    offs = np.arange(0, (n + 1) * klen, klen, dtype=np.uint64)
    return out.reshape(-1).copy(), offs


def concat(*sets):
    """Concatenate (buf, offs) key sets."""
    bufs, offs, base = [], [np.zeros(1, dtype=np.uint64)], 0
    for b, o in sets:
        bufs.append(b)
        offs.append(o[1:] - o[0] + np.uint64(base))
        base += int(o[-1] - o[0])
    return np.concatenate(bufs) if bufs else np.zeros(0, np.uint8), np.concatenate(offs)


def take(keys, idx):
    """Sub-list of a key set, in the order of idx."""
    buf, offs = keys
    parts = [buf[int(offs[i]):int(offs[i + 1])] for i in idx]
    lens = np.array([p.size for p in parts], dtype=np.uint64)
    o = np.zeros(len(parts) + 1, dtype=np.uint64)
    o[1:] = np.cumsum(lens)
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), o
