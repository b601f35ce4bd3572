"""SSTable block compression (port::Snappy_* of lsbm, i.e. libsnappy's raw
format) on the GPU.

Thin wrappers over include/lsbm_snappy.h.  Device tensors in, device tensors
out; every call enqueues on `stream` (default: torch's current stream).

    max_compressed_length(n)           snappy::MaxCompressedLength
    compress(data, offsets)            RawCompress of every block, one launch
                                       (TableBuilder::WriteBlock's call,
                                       table/table_builder.cc:186)
    uncompressed_length(data, offsets) GetUncompressedLength of every block
                                       (ReadBlock, table/format.cc:126)
    uncompress(data, offsets, ...)     RawUncompress of every block
                                       (ReadBlock, table/format.cc:130)
    keep_compressed(raw_len, comp_len) WriteBlock's 12.5% rule
                                       (table/table_builder.cc:187-188)

Blocks are a uint8 buffer plus int64 offsets (block i = data[off[i], off[i+1])).
"""
from ._lib import check, lib
from .engine import _ptr, _require_cuda, _stream_ptr, _torch

# The most a snappy stream of c bytes can expand to: a 3-byte copy tag emits
# at most 64 bytes (21.3x).  A preamble claiming more cannot be met, so
# RawUncompress fails the block; it gets no output window (uncompress()).
MAX_EXPANSION = 22


def _check(n_plus_1=None, **ts):
    """dtype / layout checks for the tensors a kernel will read or write."""
    torch = _torch()
    want = {"data": torch.uint8, "out": torch.uint8, "ok": torch.uint8, "offsets": torch.int64,
            "out_offsets": torch.int64, "out_len": torch.int64, "n_bad": torch.int32}
    for name, t in ts.items():
        if t is None:
            continue
        if t.dtype != want[name]:
            raise ValueError(f"{name} must be {want[name]}, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if n_plus_1 is not None and ts.get("out_offsets") is not None and ts["out_offsets"].numel() != n_plus_1:
        raise ValueError("out_offsets must have n + 1 entries")


def max_compressed_length(n):
    return int(lib().lsbm_snappy_max_compressed_length(int(n)))


def compress(data, offsets, out=None, out_offsets=None, out_len=None, stream=None):
    """Compress every block.  Returns (out, out_offsets, out_len): block i's
    compressed bytes are out[out_offsets[i], out_offsets[i] + out_len[i]).
    out_offsets defaults to the running sum of max_compressed_length."""
    torch = _torch()
    _require_cuda(data, offsets, out, out_offsets, out_len)
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets needs n + 1 entries")
    _check(n + 1, data=data, offsets=offsets, out=out, out_offsets=out_offsets, out_len=out_len)
    if out_len is not None and out_len.numel() < n:
        raise ValueError("out_len needs one entry per block")
    if out_offsets is None:
        lens = offsets[1:] - offsets[:-1]
        caps = 32 + lens + lens // 6
        out_offsets = torch.zeros(n + 1, dtype=torch.int64, device=offsets.device)
        torch.cumsum(caps, 0, out=out_offsets[1:])
    if out is None:
        total = int(out_offsets[-1].item()) if n else 0
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=data.device)
    if out_len is None:
        out_len = torch.empty(max(n, 1), dtype=torch.int64, device=data.device)
    check(lib().lsbm_snappy_compress_dev(_ptr(data), _ptr(offsets), n, _ptr(out), _ptr(out_offsets),
                                         _ptr(out_len), _stream_ptr(stream)),
          "lsbm_snappy_compress_dev")
    return out, out_offsets, out_len[:n]


def uncompressed_length(data, offsets, stream=None):
    """(ulen, ok) per block: GetUncompressedLength."""
    torch = _torch()
    _require_cuda(data, offsets)
    _check(data=data, offsets=offsets)
    n = offsets.numel() - 1
    ulen = torch.empty(max(n, 1), dtype=torch.int64, device=data.device)
    ok = torch.empty(max(n, 1), dtype=torch.uint8, device=data.device)
    check(lib().lsbm_snappy_uncompressed_length_dev(_ptr(data), _ptr(offsets), n, _ptr(ulen),
                                                    _ptr(ok), _stream_ptr(stream)),
          "lsbm_snappy_uncompressed_length_dev")
    return ulen[:n], ok[:n]


def uncompress(data, offsets, out=None, out_offsets=None, ok=None, n_bad=None, stream=None):
    """RawUncompress every block.  Returns (out, out_offsets, ok, n_bad):
    block i's output is out[out_offsets[i], out_offsets[i+1]), ok[i] = 1 on
    success.  Without out_offsets the lengths come from the preambles (one
    device -> host read of the total, as ReadBlock sizes its buffer)."""
    torch = _torch()
    _require_cuda(data, offsets, out, out_offsets, ok, n_bad)
    n = offsets.numel() - 1
    _check(n + 1, data=data, offsets=offsets, out=out, out_offsets=out_offsets, ok=ok, n_bad=n_bad)
    if ok is not None and ok.numel() < n:
        raise ValueError("ok needs one entry per block")
    if out_offsets is None:
        ulen, len_ok = uncompressed_length(data, offsets, stream)
        # no window for a block whose preamble cannot be met (it fails anyway)
        clen = offsets[1:] - offsets[:-1]
        ulen = torch.where((len_ok != 0) & (ulen <= MAX_EXPANSION * clen), ulen, torch.zeros_like(ulen))
        out_offsets = torch.zeros(n + 1, dtype=torch.int64, device=data.device)
        torch.cumsum(ulen, 0, out=out_offsets[1:])
    if out is None:
        total = int(out_offsets[-1].item()) if n else 0
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=data.device)
    if ok is None:
        ok = torch.empty(max(n, 1), dtype=torch.uint8, device=data.device)
    if n_bad is None:
        n_bad = torch.zeros(1, dtype=torch.int32, device=data.device)
    check(lib().lsbm_snappy_uncompress_dev(_ptr(data), _ptr(offsets), n, _ptr(out),
                                           _ptr(out_offsets), _ptr(ok), _ptr(n_bad),
                                           _stream_ptr(stream)),
          "lsbm_snappy_uncompress_dev")
    return out, out_offsets, ok[:n], n_bad


def keep_compressed(raw_len, comp_len):
    """TableBuilder::WriteBlock keeps the snappy form only when it saves at
    least 1/8: compressed < raw - raw / 8 (table/table_builder.cc:187-188)."""
    return comp_len < raw_len - raw_len // 8
