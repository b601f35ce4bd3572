#!/usr/bin/env python3
"""SSTable trailer schedules A/B inside ONE process (round 6): claimed
equal-count pieces (lsbm_test_sst_pieces(1), the default) against one range
per wave (0), alternated over the same 1M x 4,118-B image, so that the
image's physical placement -- which moved separate processes' rates by 1-2
points on one box -- is the same for both.

    python tools/ab/sst_pieces_inproc.py [--passes 8] [--reps 20]

One JSON line per pass and schedule (verify and dense trailer CRCs, HIP
events, % of 8 TB/s over block || type), then the medians.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from bench_configs import time_launches  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--passes", type=int, default=8)
    p.add_argument("--reps", type=int, default=20)
    args = p.parse_args()
    import torch
    from lsbm_amd import engine, table
    from lsbm_amd._lib import lib
    torch.cuda.set_device(0)
    engine.init(0)
    n, L = 1 << 20, 4118
    offs = np.arange(n + 1, dtype=np.int64) * (L + 5)
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0005)
    handles = torch.from_numpy(np.stack([offs[:-1], np.full(n, L, dtype=np.int64)], 1).reshape(-1).copy()).to("cuda")
    types = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    table.seal_blocks(d, handles, types, stream=s)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    nb = torch.zeros(1, dtype=torch.int32, device="cuda")
    alg = n * (L + 1)
    pct = lambda t: round(100 * alg / t / 8e12, 2)
    entries = {"sst_verify": lambda: table.verify_blocks(d, handles, stream=s),
               "sst_crcs": lambda: table.trailer_crcs(d, handles, types, stream=s, out=out, nbad=nb)}
    res = {}
    ref = None
    for ps in range(args.passes):
        for on in ((1, 0) if ps % 2 == 0 else (0, 1)):
            assert lib().lsbm_test_sst_pieces(on) == 0
            for name, fn in entries.items():
                t = time_launches(fn, s, reps=args.reps)
                res.setdefault((name, on), []).append(pct(t))
                print(json.dumps({"pass": ps, "entry": name, "pieces": on, "pct_hbm": pct(t)}), flush=True)
            ok, nbad = table.verify_blocks(d, handles, stream=s)
            assert bool(ok.all().item()) and int(nbad.item()) == 0
            table.trailer_crcs(d, handles, types, stream=s, out=out, nbad=nb)
            crcs = out.cpu().numpy()
            if ref is None:
                ref = crcs
            assert np.array_equal(crcs, ref)
    lib().lsbm_test_sst_pieces(-1)
    for (name, on), v in sorted(res.items()):
        print(json.dumps({"entry": name, "pieces": on, "median": float(np.median(v)), "all": v}), flush=True)


if __name__ == "__main__":
    main()
