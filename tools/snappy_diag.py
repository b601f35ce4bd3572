#!/usr/bin/env python3
"""A/B of the snappy decode kernel against diagnostic builds (build/diag/*.so,
snappy_kernels.hip compiled with LSBM_SNAP_DIAG_* macros; results of those
builds are wrong by design).  Times lsbm_snappy_uncompress_dev over 262,144
db_bench-shaped blocks with HIP events, interleaved, for each library."""
import ctypes
import glob
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from bench_snappy import pool_blocks  # noqa: E402

libs = {"product": ctypes.CDLL(os.path.join(REPO, "lsbm_amd", "liblsbm_crc32c.so"))}
for p in sorted(glob.glob(os.path.join(REPO, "build", "diag", "*.so"))):
    libs[os.path.basename(p)] = ctypes.CDLL(p)
P = libs["product"]
pool = pool_blocks(4096)
reps = 64
raw = b"".join(pool) * reps
lens = np.array([len(b) for b in pool] * reps, np.int64)
offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
n = len(lens)
caps = 32 + lens + lens // 6
coffs_cap = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
d = torch.from_numpy(np.frombuffer(raw, np.uint8).copy()).cuda()
o = torch.from_numpy(offs).cuda()
oc = torch.from_numpy(coffs_cap).cuda()
comp = torch.empty(int(coffs_cap[-1]), dtype=torch.uint8, device="cuda")
clen = torch.empty(n, dtype=torch.int64, device="cuda")
vp = lambda t: ctypes.c_void_p(t.data_ptr())
assert P.lsbm_snappy_compress_dev(vp(d), vp(o), ctypes.c_uint64(n), vp(comp), vp(oc), vp(clen), None) == 0
torch.cuda.synchronize()
cl = clen.cpu().numpy()
cc = comp.cpu().numpy()
packed = np.concatenate([cc[coffs_cap[i]:coffs_cap[i] + cl[i]] for i in range(n)])
co = torch.from_numpy(np.concatenate([[0], np.cumsum(cl)]).astype(np.int64)).cuda()
cd = torch.from_numpy(packed).cuda()
out = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
ok = torch.empty(n, dtype=torch.uint8, device="cuda")


def run(L):
    assert L.lsbm_snappy_uncompress_dev(vp(cd), vp(co), ctypes.c_uint64(n), vp(out), vp(o), vp(ok), None, None) == 0


res = {k: [] for k in libs}
for it in range(5):
    for k, L in libs.items():
        run(L)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(L)
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 5)
for k, v in res.items():
    print("%-28s decode %.3f ms (min of 5 rounds), %.1f GB/s raw" % (k, min(v), offs[-1] / min(v) / 1e6))
