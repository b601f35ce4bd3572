#!/usr/bin/env python3
"""Encoder phase timing from the diagnostic build (build/stamps/liblsbm_snap_stamps.so,
snappy_kernels.hip compiled with -DLSBM_SNAP_STAMPS): s_memtime cycles per block
in each phase of snappy_compress_kernel (summed over waves, per block), over db_bench-shaped data blocks."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from bench_snappy import pool_blocks  # noqa: E402

L = ctypes.CDLL(os.path.join(REPO, "build", "stamps", "liblsbm_snap_stamps.so"))
blocks = pool_blocks(4096)
data = np.frombuffer(b"".join(blocks), np.uint8)
lens = np.array([len(b) for b in blocks], np.int64)
offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
caps = 32 + lens + lens // 6
ooffs = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
d = torch.from_numpy(data).cuda()
o = torch.from_numpy(offs).cuda()
oo = torch.from_numpy(ooffs).cuda()
out = torch.empty(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
ol = torch.empty(len(blocks), dtype=torch.int64, device="cuda")
st = (ctypes.c_ulonglong * 16)()
for rep in range(3):
    L.lsbm_snappy_debug_stamps(st, 1)
    rc = L.lsbm_snappy_compress_dev(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                                    ctypes.c_uint64(len(blocks)), ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(oo.data_ptr()), ctypes.c_void_p(ol.data_ptr()), None)
    torch.cuda.synchronize()
    assert rc == 0, rc
    L.lsbm_snappy_debug_stamps(st, 0)
    nb = len(blocks)
    names = ["stage+zero", "search: match/table update", "emit_literal", "match+emit_copy", "post-copy probe",
             "remainder", "search: probe loads+buckets", "search: m0 + peer walk"]
    tot = sum(st[k] for k in range(8))
    print("rep %d waves %d blocks %d  memtime ticks/block %.0f  " % (rep, st[9], nb, tot / nb) +
          "  ".join("%s %.0f (%.0f%%)" % (names[k], st[k] / nb, 100.0 * st[k] / tot) for k in range(8)))

# decoder phases over the compressed blocks
nc = ol.cpu().numpy()
comp = out.cpu().numpy()
cblocks = [comp[int(ooffs[i]):int(ooffs[i]) + int(nc[i])].tobytes() for i in range(len(blocks))]
cdata = np.frombuffer(b"".join(cblocks), np.uint8)
coffs = np.concatenate([[0], np.cumsum([len(c) for c in cblocks])]).astype(np.int64)
cd = torch.from_numpy(cdata.copy()).cuda()
co = torch.from_numpy(coffs).cuda()
dout = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
okd = torch.empty(len(blocks), dtype=torch.uint8, device="cuda")
for rep in range(3):
    L.lsbm_snappy_debug_stamps(st, 1)
    rc = L.lsbm_snappy_uncompress_dev(ctypes.c_void_p(cd.data_ptr()), ctypes.c_void_p(co.data_ptr()),
                                      ctypes.c_uint64(len(blocks)), ctypes.c_void_p(dout.data_ptr()),
                                      ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(okd.data_ptr()), None, None)
    torch.cuda.synchronize()
    assert rc == 0, rc
    assert bool((okd == 1).all()) and torch.equal(dout, d)
    L.lsbm_snappy_debug_stamps(st, 0)
    names = ["offsets+preamble", "stage", "decode", "unstage"]
    tot = sum(st[10 + k] for k in range(4))
    print("decode rep %d waves %d blocks %d  ticks/block %.0f  " % (rep, st[15], nb, tot / nb) +
          "  ".join("%s %.0f (%.0f%%)" % (names[k], st[10 + k] / nb, 100.0 * st[10 + k] / tot) for k in range(4)))
