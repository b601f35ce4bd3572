"""Diagnostic: the SST random-layout round trip, printing every failing block."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import Oracle  # noqa: E402
from golden.splitmix import stream_bytes  # noqa: E402
from lsbm_amd import engine, table  # noqa: E402

o = Oracle(os.path.join(REPO, "oracle", "liboracle_crc32c.so"))
engine.init(0)
for seed, nblk, smax in [(21, 3000, 9000), (22, 3000, 9000), (23, 3000, 5000), (24, 3000, 2000)]:
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, smax, size=nblk)
    handles, total = table.layout_blocks(sizes)
    img = stream_bytes(seed, 0, total)
    types = rng.integers(0, 2, size=nblk).astype(np.uint8)
    d = torch.from_numpy(img).to("cuda")
    dh = torch.from_numpy(handles.astype(np.int64)).to("cuda")
    table.seal_blocks(d, dh, torch.from_numpy(types).to("cuda"))
    out = d.cpu().numpy()
    bad_seal = []
    for i in range(nblk):
        off, n = int(handles[2 * i]), int(sizes[i])
        crc = o.extend(o.value(out[off:off + n].tobytes()), bytes([types[i]]))
        if out[off + n] != types[i] or int.from_bytes(out[off + n + 1:off + n + 5].tobytes(), "little") != o.mask(crc):
            bad_seal.append(i)
    ok, nbad = table.verify_blocks(d, dh)
    okh = ok.cpu().numpy()
    bad_ver = np.nonzero(okh == 0)[0].tolist()
    print(f"seed {seed}: seal bad {len(bad_seal)} {bad_seal[:10]}  verify bad {int(nbad.item())} {bad_ver[:10]}")
    for i in sorted(set(bad_seal) | set(bad_ver))[:10]:
        off, n = int(handles[2 * i]), int(sizes[i])
        s = d.data_ptr() + off
        print(f"   blk {i} n {n} off {off} s%128 {s % 128} rows_v {((s + n + 1 + 127) >> 7) - ((s - 4) >> 7)}"
              f" rows_s {((s + n + 127) >> 7) - ((s - 4) >> 7)} type {types[i]}"
              f" prev_n {sizes[i-1] if i else -1} next_n {sizes[i+1] if i + 1 < nblk else -1}")
    # ragged kModeOut over the same block||type extents, vs oracle
    ext = np.stack([handles[0::2], handles[1::2] + 1], 1).reshape(-1).astype(np.int64)
    got = engine.crc32c_extents(d, torch.from_numpy(ext).to("cuda")).cpu().numpy().view(np.uint32)
    bad_ext = [i for i in range(nblk) if got[i] != o.value(out[int(handles[2*i]):int(handles[2*i]) + int(sizes[i]) + 1].tobytes())]
    print(f"   extents-mode mismatches {len(bad_ext)} {bad_ext[:10]}")
