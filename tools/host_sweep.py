#!/usr/bin/env python3
"""Host-staged rate vs staging chunk size (one subprocess per size, since the
engine reads LSBM_STAGE_CHUNK_MB once).  Prints one JSON line per size."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, time, numpy as np, torch
sys.path.insert(0, %r)
from lsbm_amd import engine
torch.cuda.set_device(0); engine.init(0)
n, L = 1 << 18, 4096
src = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
d = torch.empty(n * L, dtype=torch.uint8, device="cuda"); engine.fill_splitmix64(d, 0x5EED0000)
src.copy_(d); h = src.numpy()
offs = np.arange(0, (n + 1) * L, L, dtype=np.uint64)
ref = engine.crc32c_fixed(d, L, L, n).cpu().numpy().view(np.uint32)
engine.crc32c_batch_host(h, offs)
t0 = time.perf_counter()
for _ in range(5): got = engine.crc32c_batch_host(h, offs)
el = (time.perf_counter() - t0) / 5
print(json.dumps({"chunk_mb": int(sys.argv[1]), "GBps": round(n * L / el / 1e9, 2),
                  "bad": int((got != ref).sum())}))
''' % REPO

for mb in (int(x) for x in (sys.argv[1:] or ["16", "32", "64", "128", "256"])):
    env = dict(os.environ, LSBM_STAGE_CHUNK_MB=str(mb))
    r = subprocess.run([sys.executable, "-c", CHILD, str(mb)], env=env, capture_output=True,
                       text=True, timeout=300)
    print(r.stdout.strip() or r.stderr[-500:], flush=True)
    if r.returncode:
        sys.exit(r.returncode)
