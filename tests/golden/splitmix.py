"""Seeded byte streams shared by the golden-vector generator and the tests.

Stream definition: 8-byte word w of a stream with seed s is
splitmix64(s + w), stored little-endian; byte a of the stream is byte (a % 8)
of word (a // 8).  numpy uint64 arithmetic wraps modulo 2**64, as required.
"""
import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + _G
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
    return x ^ (x >> np.uint64(31))


def stream_bytes(seed, byte_off, nbytes):
    """Bytes [byte_off, byte_off + nbytes) of the stream for `seed` (np.uint8)."""
    if nbytes == 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = byte_off // 8
    w1 = (byte_off + nbytes + 7) // 8
    with np.errstate(over="ignore"):
        words = splitmix64(np.uint64(seed) + np.arange(w0, w1, dtype=np.uint64))
    raw = words.astype("<u8").view(np.uint8)
    s = byte_off - w0 * 8
    return raw[s:s + nbytes].copy()


def printable_bytes(seed, nbytes):
    """db_bench-like printable payload (' '..'~', util/testutil.cc:12-18)."""
    b = stream_bytes(seed, 0, nbytes)
    return (np.uint8(32) + (b % np.uint8(95))).astype(np.uint8)
