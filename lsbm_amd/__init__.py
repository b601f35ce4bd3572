"""lsbm_amd -- MI355X-native batched CRC-32C engine for lsbm's block checksums.

  lsbm_amd.crc32c   util/crc32c.h mirror (Value / Extend / Mask / Unmask)
  lsbm_amd.engine   device-resident and host-staged batches (GPU)
  lsbm_amd.table    SSTable block trailers: batched WriteRawBlock / ReadBlock verify
  lsbm_amd.log      WAL / MANIFEST record CRCs: batched log::Writer seal / log::Reader check
  lsbm_amd.bloom    SSTable bloom filters: batched CreateFilter / KeyMayMatch / filter blocks
  lsbm_amd.snappy   SSTable block compression: batched snappy RawCompress / RawUncompress

The compute lives in lsbm_amd/liblsbm_crc32c.so (hand-written gfx950 HIP
kernels behind the C ABIs in include/lsbm_crc32c.h, include/lsbm_bloom.h and include/lsbm_snappy.h).
"""
from ._lib import LIB_PATH, LsbmError, lib  # noqa: F401

__all__ = ["LIB_PATH", "LsbmError", "lib", "crc32c", "engine", "table", "log", "bloom", "snappy"]
