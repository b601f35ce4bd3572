"""Batched CRC-32C on the GPU: thin Python wrappers over include/lsbm_crc32c.h.

All tensors are device tensors (torch is only device-memory / stream
plumbing); every call enqueues on `stream` (default: torch's current stream)
and returns without synchronising.  Nothing here computes on the CPU.

  crc32c_fixed(data, stride, length, n_blocks)   lsbm_crc32c_fixed_dev
  crc32c_batch(data, offsets)                    lsbm_crc32c_batch_dev
  crc32c_extents(data, extents)                  lsbm_crc32c_extents_dev
  crc32c_verify(data, offsets, expect)           lsbm_crc32c_verify_dev
  crc32c_batch_host(data_np, offsets_np)         lsbm_crc32c_batch_host
  fill_splitmix64(buf, seed), stream_read(buf)   benchmark helpers

Each block's result equals crc32c::Extend(init[i] or 0, block_i, n_i)
(util/crc32c.cc:286-329), Mask()ed when masked=True (util/crc32c.h:31-34).
"""
import ctypes

import numpy as np

from ._lib import LSBM_CRC32C_MASKED, check, lib


def _torch():
    import torch  # noqa: WPS433 (plumbing only)
    return torch


def _stream_ptr(stream):
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("device tensors required (use crc32c_batch_host for host data)")


def init(device=0):
    check(lib().lsbm_crc32c_init(int(device)), "lsbm_crc32c_init")


def crc32c_fixed(data, stride, length, n_blocks, init=None, masked=False, out=None,
                 stream=None):
    """Block i = data[i*stride : i*stride+length] (uint8 device tensor)."""
    torch = _torch()
    _require_cuda(data, init, out)
    if n_blocks and (n_blocks - 1) * stride + length > data.numel():
        raise ValueError("blocks extend past the end of `data`")
    if init is not None and init.numel() < n_blocks:
        raise ValueError("init must have n_blocks entries")
    if out is None:
        out = torch.empty(n_blocks, dtype=torch.int32, device=data.device)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_fixed_dev(_ptr(data), stride, length, n_blocks, _ptr(init),
                                      _ptr(out), flags, _stream_ptr(stream)),
          "lsbm_crc32c_fixed_dev")
    return out


def _check_offsets(data, offsets):
    if offsets.dtype != _torch().int64:
        raise ValueError("offsets must be int64")
    return offsets.numel() - 1


def crc32c_batch(data, offsets, init=None, masked=False, out=None, stream=None):
    """Block i = data[offsets[i] : offsets[i+1]] (offsets: int64 device tensor)."""
    torch = _torch()
    _require_cuda(data, offsets, init, out)
    n = _check_offsets(data, offsets)
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int32, device=data.device)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_batch_dev(_ptr(data), _ptr(offsets), max(n, 0), _ptr(init),
                                      _ptr(out), flags, _stream_ptr(stream)),
          "lsbm_crc32c_batch_dev")
    return out


def crc32c_extents(data, extents, init=None, masked=False, out=None, stream=None):
    """Block i = data[ext[2i] : ext[2i] + ext[2i+1]] (int64 {offset, length} pairs)."""
    torch = _torch()
    _require_cuda(data, extents, init, out)
    if extents.dtype != torch.int64 or extents.numel() % 2:
        raise ValueError("extents must be int64 {offset, length} pairs")
    n = extents.numel() // 2
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_extents_dev(_ptr(data), _ptr(extents), n, _ptr(init), _ptr(out),
                                        flags, _stream_ptr(stream)),
          "lsbm_crc32c_extents_dev")
    return out


def crc32c_verify(data, offsets, expect, init=None, masked=False, stream=None):
    """Returns (ok uint8[n], nbad int32[1]) device tensors."""
    torch = _torch()
    _require_cuda(data, offsets, expect, init)
    n = _check_offsets(data, offsets)
    ok = torch.empty(max(n, 0), dtype=torch.uint8, device=data.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=data.device)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_verify_dev(_ptr(data), _ptr(offsets), max(n, 0), _ptr(init),
                                       _ptr(expect), _ptr(ok), _ptr(nbad), flags,
                                       _stream_ptr(stream)),
          "lsbm_crc32c_verify_dev")
    return ok, nbad


def crc32c_batch_host(data, offsets, init=None, masked=False, device=0):
    """Host-staged batch: numpy uint8 data + uint64/int64 offsets -> numpy uint32."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty(max(n, 0), dtype=np.uint32)
    if init is not None:
        init = np.ascontiguousarray(init, dtype=np.uint32)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_batch_host(int(device), data.ctypes.data_as(ctypes.c_void_p),
                                       offsets.ctypes.data_as(ctypes.c_void_p), max(n, 0),
                                       init.ctypes.data_as(ctypes.c_void_p) if init is not None
                                       else None,
                                       out.ctypes.data_as(ctypes.c_void_p), flags),
          "lsbm_crc32c_batch_host")
    return out


def crc32c_batch_host_multi(data, offsets, devices, init=None, masked=False):
    """crc32c_batch_host sharded over `devices` (one host thread per device,
    contiguous shards of about equal bytes, no collective)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty(max(n, 0), dtype=np.uint32)
    if init is not None:
        init = np.ascontiguousarray(init, dtype=np.uint32)
    devs = (ctypes.c_int * len(devices))(*devices)
    flags = LSBM_CRC32C_MASKED if masked else 0
    check(lib().lsbm_crc32c_batch_host_multi(devs, len(devices), data.ctypes.data_as(ctypes.c_void_p),
                                             offsets.ctypes.data_as(ctypes.c_void_p), max(n, 0),
                                             init.ctypes.data_as(ctypes.c_void_p) if init is not None
                                             else None, out.ctypes.data_as(ctypes.c_void_p), flags),
          "lsbm_crc32c_batch_host_multi")
    return out


def fill_splitmix64(buf, seed, stream=None):
    """buf[k] = byte k of the splitmix64 stream `seed` (uint8 device tensor)."""
    _require_cuda(buf)
    check(lib().lsbm_fill_splitmix64_dev(_ptr(buf), buf.numel(), seed & (2**64 - 1),
                                         _stream_ptr(stream)),
          "lsbm_fill_splitmix64_dev")
    return buf


def stream_read(buf, sink, stream=None):
    _require_cuda(buf, sink)
    check(lib().lsbm_stream_read_dev(_ptr(buf), buf.numel(), _ptr(sink), _stream_ptr(stream)),
          "lsbm_stream_read_dev")


def as_u32(t):
    """int32 result tensor -> numpy uint32 (host copy)."""
    return t.cpu().numpy().view(np.uint32)
