import sys, os, json, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, 'tools')
from bench_configs import time_launches
from lsbm_amd import engine, table
engine.init(0)
n, S = 1 << 20, 4123
d = torch.empty(n * S + 64, dtype=torch.uint8, device="cuda")
engine.fill_splitmix64(d, 5)
s = torch.cuda.current_stream()
out = torch.empty(n, dtype=torch.int32, device="cuda")
offs = np.arange(n, dtype=np.int64) * S
for L in (4096, 4110, 4117, 4118, 4119, 4120, 4123):
    ext = torch.from_numpy(np.stack([offs, np.full(n, L)], 1).reshape(-1).copy()).to("cuda")
    t = time_launches(lambda: engine.crc32c_extents(d, ext, out=out, stream=s), s, reps=10)
    hs = torch.from_numpy(np.stack([offs, np.full(n, L - 1 if L > 0 else 0)], 1).reshape(-1).copy()).to("cuda")
    types = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tt = time_launches(lambda: table.trailer_crcs(d, hs, types, stream=s, out=out), s, reps=10)
    print(L, "ext %.2f%%" % (100 * n * L / t / 8e12), "tcrc(n=L-1) %.2f%%" % (100 * n * (L - 1) / tt / 8e12), flush=True)
