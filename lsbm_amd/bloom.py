"""SSTable bloom filters (util/bloom.cc, table/filter_block.cc of lsbm) on the GPU.

Thin wrappers over include/lsbm_bloom.h.  Device tensors in, device tensors
out; every call enqueues on `stream` (default: torch's current stream).

    hash(data, seed)                  leveldb::Hash (util/hash.cc:18-49), host
    filter_bytes / k_build / k_probe  BloomFilterPolicy's size and probe rules
    build_filters(...)                CreateFilter for many filters (one launch)
    may_match(...)                    KeyMayMatch for many lookups
    filter_block_may_match(...)       FilterBlockReader::KeyMayMatch, batched
    layout_filter_block(...)          FilterBlockBuilder's layout (host)
    build_filter_block(...)           a whole FilterBlockBuilder::Finish result

Keys are a uint8 buffer plus int64 offsets (key i = keys[off[i], off[i+1]));
strip=8 drops the internal-key suffix first, as InternalFilterPolicy does
(common/dbformat.cc:105-119).
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._lib import check, lib
from .engine import _ptr, _require_cuda, _stream_ptr, _torch

kFilterBaseLg = 11  # table/filter_block.cc:15
kFilterBase = 1 << kFilterBaseLg
BLOOM_SEED = 0xBC9F1D34  # util/bloom.cc:14


def hash(data, seed=BLOOM_SEED):  # noqa: A001 (the reference's name)
    b = bytes(data)
    return lib().lsbm_bloom_hash(ctypes.c_char_p(b), len(b), seed & 0xFFFFFFFF)


def filter_bytes(n_keys, bits_per_key):
    return int(lib().lsbm_bloom_filter_bytes(int(n_keys), int(bits_per_key)))


def k_build(bits_per_key):
    return int(lib().lsbm_bloom_k(int(bits_per_key)))


def k_probe(bits_per_key, bloom_bits_use=15):
    return int(lib().lsbm_bloom_k_probe(int(bits_per_key), int(bloom_bits_use)))


def build_filters(keys, key_offsets, filter_first, filter_out, out, bits_per_key, strip=0,
                  stream=None):
    """Filter f of keys [filter_first[f], filter_first[f+1]) -> out[filter_out[f], ...)."""
    _require_cuda(keys, key_offsets, filter_first, filter_out, out)
    n = filter_out.numel()
    if filter_first.numel() != n + 1:
        raise ValueError("filter_first needs n_filters + 1 entries")
    check(lib().lsbm_bloom_build_dev(_ptr(keys), _ptr(key_offsets), strip, _ptr(filter_first),
                                     _ptr(filter_out), n, bits_per_key, _ptr(out),
                                     _stream_ptr(stream)), "lsbm_bloom_build_dev")
    return out


def _probe_out(n, device, may, n_may):
    """Result tensors: given ones are reused (n_may accumulates), else new."""
    torch = _torch()
    if may is None:
        may = torch.empty(n, dtype=torch.uint8, device=device)
    if n_may is None:
        n_may = torch.zeros(1, dtype=torch.int32, device=device)
    if may.numel() < n:
        raise ValueError("may needs one byte per query")
    return may, n_may


def may_match(filters, handles, keys, key_offsets, bits_per_key, bloom_bits_use=15, strip=0,
              stream=None, may=None, n_may=None):
    """Query q: key q against filters[handles[2q], + handles[2q+1]).
    Returns (may uint8[n], n_may int32[1]); the count is added to a given n_may."""
    _require_cuda(filters, handles, keys, key_offsets)
    n = key_offsets.numel() - 1
    may, n_may = _probe_out(n, filters.device, may, n_may)
    check(lib().lsbm_bloom_may_match_dev(_ptr(filters), _ptr(handles), _ptr(keys),
                                         _ptr(key_offsets), strip, n, bits_per_key,
                                         bloom_bits_use, _ptr(may), _ptr(n_may),
                                         _stream_ptr(stream)), "lsbm_bloom_may_match_dev")
    return may, n_may


def filter_block_may_match(blocks, handles, data_offsets, keys, key_offsets, bits_per_key,
                           bloom_bits_use=15, strip=0, stream=None, may=None, n_may=None):
    """Query q: FilterBlockReader(blocks[handles[2q], + handles[2q+1]])
    .KeyMayMatch(data_offsets[q], key q).  Returns (may, n_may)."""
    _require_cuda(blocks, handles, data_offsets, keys, key_offsets)
    n = key_offsets.numel() - 1
    may, n_may = _probe_out(n, blocks.device, may, n_may)
    check(lib().lsbm_filter_block_may_match_dev(_ptr(blocks), _ptr(handles), _ptr(data_offsets),
                                                _ptr(keys), _ptr(key_offsets), strip, n,
                                                bits_per_key, bloom_bits_use, _ptr(may),
                                                _ptr(n_may), _stream_ptr(stream)),
          "lsbm_filter_block_may_match_dev")
    return may, n_may


@dataclass
class FilterBlockLayout:
    filter_keys: list = field(default_factory=list)   # (k0, k1) of each non-empty filter
    filter_out: list = field(default_factory=list)    # its byte offset in the block
    offsets: list = field(default_factory=list)       # the offset array (one per filter)
    data_bytes: int = 0
    trailer: bytes = b""                              # offsets + array_offset + base_lg

    @property
    def total_bytes(self):
        return self.data_bytes + len(self.trailer)


def layout_filter_block(block_start, block_first, bits_per_key):
    """FilterBlockBuilder for the sequence StartBlock(block_start[b]), AddKey
    for keys [block_first[b], block_first[b+1]), ..., Finish()
    (table/filter_block.cc:22-76): which keys form which filter, and where."""
    lay = FilterBlockLayout()
    n_blocks = len(block_start)
    lo = hi = int(block_first[0]) if n_blocks else 0

    def generate():
        nonlocal lo
        lay.offsets.append(lay.data_bytes)
        if hi > lo:
            lay.filter_keys.append((lo, hi))
            lay.filter_out.append(lay.data_bytes)
            lay.data_bytes += filter_bytes(hi - lo, bits_per_key)
            lo = hi

    for b in range(n_blocks):
        while int(block_start[b]) // kFilterBase > len(lay.offsets):
            generate()
        hi = int(block_first[b + 1])
    if hi > lo:
        generate()
    tr = b"".join(int(o).to_bytes(4, "little") for o in lay.offsets)
    lay.trailer = tr + int(lay.data_bytes).to_bytes(4, "little") + bytes([kFilterBaseLg])
    return lay


def build_filter_block(keys, key_offsets, block_start, block_first, bits_per_key, strip=0,
                       stream=None):
    """The bytes FilterBlockBuilder::Finish returns, every filter computed in
    one launch (keys / key_offsets: device tensors)."""
    torch = _torch()
    lay = layout_filter_block(block_start, block_first, bits_per_key)
    data = b""
    if lay.filter_keys:
        dev = keys.device
        first = torch.tensor([k0 for k0, _ in lay.filter_keys] + [lay.filter_keys[-1][1]],
                             dtype=torch.int64, device=dev)
        outo = torch.tensor(lay.filter_out, dtype=torch.int64, device=dev)
        out = torch.empty(max(1, lay.data_bytes), dtype=torch.uint8, device=dev)
        build_filters(keys, key_offsets, first, outo, out, bits_per_key, strip, stream)
        data = out[:lay.data_bytes].cpu().numpy().tobytes()
    return data + lay.trailer
