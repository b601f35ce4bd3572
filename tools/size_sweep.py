#!/usr/bin/env python3
"""The fixed kernel's rate against the batch's size and place (DESIGN.md section 6:
per-GPU rate of a config-5 shard vs config 2):

    LSBM_FIXED_SPLIT_BLOCKS=0 python tools/size_sweep.py [--gib 40]

(=0: one launch per call, as measured in round 5 before big batches were split.)

One buffer of --gib GiB of 4 KiB blocks; lsbm_crc32c_fixed_dev over sub-batches
of 1M, 2M, 4M and all blocks, at the buffer's start and end, each timed with HIP
events over 20 launches after a 0.3 s spin-up.  One JSON line per case."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=40)
    a = ap.parse_args()
    import torch
    from lsbm_amd import engine
    torch.cuda.set_device(0)
    engine.init(0)
    L = 4096
    n_all = (a.gib << 30) // L
    d = torch.empty(n_all * L, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0000)
    out = torch.empty(n_all, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for n in (1 << 20, 2 << 20, 4 << 20, n_all):
        for where in ("start", "end"):
            if n == n_all and where == "end":
                continue
            lo = 0 if where == "start" else n_all - n
            view = d[lo * L:(lo + n) * L]
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                engine.crc32c_fixed(view, L, L, n, out=out, stream=s)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record(s)
            for _ in range(reps):
                engine.crc32c_fixed(view, L, L, n, out=out, stream=s)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(json.dumps({"blocks": n, "where": where, "ms": round(ms, 4),
                              "GiBps": round(n * L / (ms / 1e3) / 2**30, 1),
                              "pct_8TBs": round(100 * n * L / (ms / 1e3) / 8e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
