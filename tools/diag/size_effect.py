"""Diagnostic: why the ragged kernel's rate falls with the batch size
(profiles/r02/ab/s58_usweep_size.log: 81% of HBM peak at 16 GiB of 12 KiB
blocks, 75% at 117 GiB).  One 117 GiB allocation of equal 12,288-B blocks,
5 bytes off alignment; timed with HIP events after a spin-up:
  part  -- the first 16 GiB of it as one batch
  split -- all of it as 7 consecutive launches of 1/7 each
  whole -- all of it as one launch
Run on the GPU box: python tools/diag/size_effect.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from lsbm_amd import engine  # noqa: E402

HBM = 8000.0


def timed(fns, s, reps=5, spin_s=0.3):
    t_end = time.perf_counter() + spin_s
    while time.perf_counter() < t_end:
        for f in fns:
            f()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        for f in fns:
            f()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / 1e3 / reps


def main():
    torch.cuda.set_device(0)
    engine.init(0)
    L = 12288
    n = (117 << 30) // L
    d = torch.empty(n * L + 4096, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0003)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda") + 5
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    np_ = (16 << 30) // L
    t = timed([lambda: engine.crc32c_batch(d, offs[:np_ + 1], out=out[:np_], stream=s)], s)
    res["part_16GiB"] = round(100 * np_ * L / t / 1e9 / HBM, 2)
    k = 7
    cuts = [n * i // k for i in range(k + 1)]
    fns = [(lambda a=a, b=b: engine.crc32c_batch(d, offs[a:b + 1], out=out[a:b], stream=s))
           for a, b in zip(cuts[:-1], cuts[1:])]
    t = timed(fns, s)
    res["split_7x"] = round(100 * n * L / t / 1e9 / HBM, 2)
    t = timed([lambda: engine.crc32c_batch(d, offs, out=out, stream=s)], s)
    res["whole"] = round(100 * n * L / t / 1e9 / HBM, 2)
    print(json.dumps({"diag": "size_effect", "block": L, "blocks": n, "pct_hbm_peak": res}), flush=True)


if __name__ == "__main__":
    main()
