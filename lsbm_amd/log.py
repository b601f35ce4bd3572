"""WAL / MANIFEST record CRCs (common/log_*.cc of lsbm), batched on the GPU.

A log image is 32 KiB blocks of physical records, each a 7-byte header
[masked crc LE32][length LE16][type u8] plus `length` payload bytes
(common/log_format.h).  The reference seals one record at a time in
log::Writer::EmitPhysicalRecord (common/log_writer.cc:75-100) and checks one
at a time in log::Reader::ReadPhysicalRecord (common/log_reader.cc:228-242);
here every header of a device-resident image is sealed / verified in one
launch.  The C++ host layer that frames records and replays the reader is
include/lsbm/log_checksum.h.
"""
import numpy as np

from ._lib import check, lib
from .engine import _ptr, _require_cuda, _stream_ptr, _torch

kBlockSize = 32768  # common/log_format.h:27
kHeaderSize = 7     # common/log_format.h:30
kZeroType, kFullType, kFirstType, kMiddleType, kLastType = range(5)


def layout_records(payloads):
    """Frame records as log::Writer::AddRecord does (common/log_writer.cc:27-73),
    CRC fields left zero.  Returns (image uint8, header offsets int64)."""
    out, heads, bo = bytearray(), [], 0
    for p in payloads:
        p = bytes(p)
        pos, first = 0, True
        while True:
            if kBlockSize - bo < kHeaderSize:
                out += bytes(kBlockSize - bo)
                bo = 0
            frag = min(len(p) - pos, kBlockSize - bo - kHeaderSize)
            last = pos + frag == len(p)
            t = (kFullType if last else kFirstType) if first else (kLastType if last else kMiddleType)
            heads.append(len(out))
            out += bytes(4) + bytes([frag & 0xFF, frag >> 8, t]) + p[pos:pos + frag]
            bo += kHeaderSize + frag
            pos += frag
            first = False
            if pos == len(p):
                break
    return np.frombuffer(bytes(out), dtype=np.uint8).copy(), np.array(heads, dtype=np.int64)


def seal_records(image, headers, stream=None):
    """lsbm_log_seal_dev: write every header's masked CRC in place.
    Returns (masked uint32-as-int32[n], nbad int32[1]) device tensors."""
    torch = _torch()
    _require_cuda(image, headers)
    n = headers.numel()
    masked = torch.empty(n, dtype=torch.int32, device=image.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=image.device)
    check(lib().lsbm_log_seal_dev(_ptr(image), image.numel(), _ptr(headers), n, _ptr(masked),
                                  _ptr(nbad), _stream_ptr(stream)), "lsbm_log_seal_dev")
    return masked, nbad


def verify_records(image, headers, stream=None):
    """lsbm_log_verify_dev: returns (ok uint8[n], nbad int32[1]) device tensors."""
    torch = _torch()
    _require_cuda(image, headers)
    n = headers.numel()
    ok = torch.empty(n, dtype=torch.uint8, device=image.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=image.device)
    check(lib().lsbm_log_verify_dev(_ptr(image), image.numel(), _ptr(headers), n, _ptr(ok),
                                    _ptr(nbad), _stream_ptr(stream)), "lsbm_log_verify_dev")
    return ok, nbad
