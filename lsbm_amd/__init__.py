"""lsbm_amd -- MI355X-native batched CRC-32C engine for lsbm's block checksums.

  lsbm_amd.crc32c   util/crc32c.h mirror (Value / Extend / Mask / Unmask)
  lsbm_amd.engine   device-resident and host-staged batches (GPU)
  lsbm_amd.table    SSTable block trailers: batched WriteRawBlock / ReadBlock verify

The compute lives in lsbm_amd/liblsbm_crc32c.so (hand-written gfx950 HIP
kernels behind the C ABI in include/lsbm_crc32c.h).
"""
from ._lib import LIB_PATH, LsbmError, lib  # noqa: F401

__all__ = ["LIB_PATH", "LsbmError", "lib", "crc32c", "engine", "table"]
