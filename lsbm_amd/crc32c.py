"""Python mirror of lsbm's util/crc32c.h API (util/crc32c.h:17-40).

    value(data)            == crc32c::Value(data, n)          (util/crc32c.h:20-22)
    extend(init_crc, data) == crc32c::Extend(init_crc, data, n) (util/crc32c.cc:286)
    mask(crc) / unmask(m)  == crc32c::Mask / Unmask            (util/crc32c.h:31-40)
    MASK_DELTA             == crc32c::kMaskDelta                (util/crc32c.h:24)

Scalar calls go to the library's host CRC (leveldb::crc32c::Extend exported by
liblsbm_crc32c.so); batches of blocks go to the GPU (lsbm_amd.engine).
"""
import ctypes

from ._lib import LSBM_CRC32C_MASK_DELTA, lib

MASK_DELTA = LSBM_CRC32C_MASK_DELTA


def _buf(data):
    if isinstance(data, str):
        data = data.encode()
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data)
        return b, len(b)
    # numpy arrays and other buffer-protocol objects
    mv = memoryview(data).cast("B")
    b = mv.tobytes()
    return b, len(b)


def extend(init_crc, data):
    b, n = _buf(data)
    return lib().lsbm_crc32c_extend(init_crc & 0xFFFFFFFF, ctypes.c_char_p(b), n)


def value(data):
    b, n = _buf(data)
    return lib().lsbm_crc32c_value(ctypes.c_char_p(b), n)


def mask(crc):
    return lib().lsbm_crc32c_mask(crc & 0xFFFFFFFF)


def unmask(masked_crc):
    return lib().lsbm_crc32c_unmask(masked_crc & 0xFFFFFFFF)
