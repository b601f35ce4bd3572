"""SSTable block-trailer boundary (table/ layer of lsbm), batched on the GPU.

The reference seals every block in TableBuilder::WriteRawBlock
(table/table_builder.cc:237-255):

    trailer = [type u8][EncodeFixed32(Mask(Extend(Value(block, n), &type, 1)))]

and ReadBlock (table/format.cc:95-103) verifies, when
ReadOptions::verify_checksums is set,

    Unmask(DecodeFixed32(data + n + 1)) == Value(data, n + 1)

returning Status::Corruption("block checksum mismatch") otherwise.  Here a
*file image* (uint8 device tensor) plus BlockHandles ({offset, size} int64
pairs, table/format.h:22-50) are sealed / verified in one launch.
"""
import ctypes

import numpy as np

from ._lib import LSBM_BLOCK_TRAILER_SIZE, check, lib
from .engine import _ptr, _require_cuda, _stream_ptr, _torch

kBlockTrailerSize = LSBM_BLOCK_TRAILER_SIZE  # table/format.h:84
kNoCompression = 0x0  # include/leveldb/options.h:27
kSnappyCompression = 0x1  # include/leveldb/options.h:28


class Status:
    """Minimal mirror of leveldb::Status (include/leveldb/status.h)."""

    def __init__(self, code="OK", msg=""):
        self.code, self.msg = code, msg

    @staticmethod
    def OK():
        return Status()

    @staticmethod
    def Corruption(msg):
        return Status("Corruption", msg)

    def ok(self):
        return self.code == "OK"

    def IsCorruption(self):
        return self.code == "Corruption"

    def ToString(self):
        return "OK" if self.ok() else f"{self.code}: {self.msg}"

    __str__ = ToString


def layout_blocks(sizes):
    """Handles for blocks written back to back, each followed by its trailer
    (offset += size + kBlockTrailerSize, table/table_builder.cc:251)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    offs = np.zeros(sizes.size, dtype=np.int64)
    if sizes.size:
        offs[1:] = np.cumsum(sizes + kBlockTrailerSize)[:-1]
    handles = np.stack([offs, sizes], axis=1).reshape(-1)
    total = int(offs[-1] + sizes[-1] + kBlockTrailerSize) if sizes.size else 0
    return handles, total


def _check_image(file_image, handles, types=None):
    torch = _torch()
    _require_cuda(file_image, handles, types)
    if file_image.dtype != torch.uint8 or not file_image.is_contiguous():
        raise ValueError("file_image must be a contiguous uint8 tensor")
    if handles.dtype != torch.int64 or handles.numel() % 2 or not handles.is_contiguous():
        raise ValueError("handles must be contiguous int64 {offset, size} pairs")
    n = handles.numel() // 2
    if types is not None and (types.dtype != torch.uint8 or types.numel() < n):
        raise ValueError("types must be uint8 with one entry per block")
    return n


def seal_blocks(file_image, handles, types, stream=None, nbad=None):
    """Batched WriteRawBlock trailers: writes file_image[off+size : off+size+5].
    Handles whose size + 5 bytes fall outside the image are left alone and
    counted into `nbad` (int32[1], returned; created when None)."""
    torch = _torch()
    n = _check_image(file_image, handles, types)
    if nbad is None:
        nbad = torch.zeros(1, dtype=torch.int32, device=file_image.device)
    check(lib().lsbm_sst_seal_dev(_ptr(file_image), file_image.numel(), _ptr(handles),
                                  _ptr(types), n, _ptr(nbad), _stream_ptr(stream)),
          "lsbm_sst_seal_dev")
    return nbad


def trailer_crcs(file_image, handles, types, stream=None, out=None, nbad=None):
    """Batched WriteRawBlock CRCs without touching the image: returns (masked
    int32[n], nbad int32[1]); masked[i] is the trailer's crc field
    Mask(Extend(Value(block i), &types[i], 1)), 0 for handles past the image."""
    torch = _torch()
    n = _check_image(file_image, handles, types)
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=file_image.device)
    if nbad is None:
        nbad = torch.zeros(1, dtype=torch.int32, device=file_image.device)
    check(lib().lsbm_sst_trailer_crcs_dev(_ptr(file_image), file_image.numel(), _ptr(handles),
                                          _ptr(types), n, _ptr(out), _ptr(nbad),
                                          _stream_ptr(stream)), "lsbm_sst_trailer_crcs_dev")
    return out, nbad


def verify_blocks(file_image, handles, stream=None):
    """Batched ReadBlock verify: returns (ok uint8[n], nbad int32[1]).  A
    handle past the image (truncated block read) is not ok."""
    torch = _torch()
    n = _check_image(file_image, handles)
    ok = torch.empty(n, dtype=torch.uint8, device=file_image.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=file_image.device)
    check(lib().lsbm_sst_verify_dev(_ptr(file_image), file_image.numel(), _ptr(handles), n,
                                    _ptr(ok), _ptr(nbad), _stream_ptr(stream)),
          "lsbm_sst_verify_dev")
    return ok, nbad


def read_block_status(ok_flag):
    """Map one verify flag to ReadBlock's status (table/format.cc:98-101)."""
    return Status.OK() if ok_flag else Status.Corruption("block checksum mismatch")


def verify_status(file_image, handles, stream=None):
    """First failing block's Status, like a sequence of ReadBlock calls."""
    ok, nbad = verify_blocks(file_image, handles, stream)
    if int(nbad.item()) == 0:
        return Status.OK(), ok
    return Status.Corruption("block checksum mismatch"), ok


_ = ctypes  # ctypes handles live in _lib
