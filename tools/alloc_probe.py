#!/usr/bin/env python3
"""The fixed kernel over one 10M-block (40 GiB) batch allocated three ways
(per-GPU rate of a config-5 shard):

    LSBM_FIXED_SPLIT_BLOCKS=0 python tools/alloc_probe.py [--blocks 10000000]

(=0: one launch per lsbm_crc32c_fixed_dev call, as the cases below assume;
the library's default splits a batch of 2M+ blocks into 1M-block launches.)

  torch       torch.empty (the caching allocator's hipMalloc), as bench.py
  hipMalloc   hipMalloc directly
  contiguous  hipExtMallocWithFlags(..., hipDeviceMallocContiguous)
  split       one torch buffer swept by launches of 512K-4M blocks
  chunks      the same blocks as 1M-block allocations, one launch each

Each: fill (splitmix64 0x5EED0000), 0.3 s spin-up, then 20 launches between
HIP events; the 1M-block batch at each buffer's start for comparison; CRCs of
the three checked equal.  One JSON line per case."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch
    from lsbm_amd import engine
    from lsbm_amd._lib import lib
    torch.cuda.set_device(0)
    engine.init(0)
    hip = ctypes.CDLL("libamdhip64.so")
    L = 4096
    n = a.blocks
    nbytes = n * L
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    lb = lib()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = None
    for how in ("torch", "hipMalloc", "contiguous"):
        keep = None
        if how == "torch":
            keep = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            ptr = keep.data_ptr()
        else:
            p = ctypes.c_void_p()
            if how == "hipMalloc":
                rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
            else:
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4))
            if rc != 0:
                print(json.dumps({"alloc": how, "error": rc}), flush=True)
                continue
            ptr = p.value
        assert lb.lsbm_fill_splitmix64_dev(ctypes.c_void_p(ptr), nbytes, 0x5EED0000, sp) == 0
        for m in (n, 1 << 20):
            def launch():
                assert lb.lsbm_crc32c_fixed_dev(ctypes.c_void_p(ptr), L, L, m, None,
                                                ctypes.c_void_p(out.data_ptr()), 0, sp) == 0
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                launch()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                launch()
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            if m == n:
                crc = out.cpu()
                same = True if ref is None else bool(torch.equal(crc, ref))
                ref = crc if ref is None else ref
            print(json.dumps({"alloc": how, "blocks": m, "ms": round(ms, 4),
                              "GiBps": round(m * L / (ms / 1e3) / 2**30, 1),
                              "pct_8TBs": round(100 * m * L / (ms / 1e3) / 8e12, 2),
                              "crcs_equal_torch": same if m == n else None}), flush=True)
        del keep
        if how != "torch":
            hip.hipFree(ctypes.c_void_p(ptr))
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    # one torch buffer, swept by launches of `per` blocks each (back to back on
    # the stream): whether the one-launch rate is the buffer or the launch
    keep = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lb.lsbm_fill_splitmix64_dev(ctypes.c_void_p(keep.data_ptr()), nbytes, 0x5EED0000, sp) == 0
    for per in (1 << 19, 1 << 20, 1 << 21, 1 << 22):
        def launch_split():
            for f in range(0, n, per):
                m = min(per, n - f)
                assert lb.lsbm_crc32c_fixed_dev(ctypes.c_void_p(keep.data_ptr() + f * L), L, L, m, None,
                                                ctypes.c_void_p(out.data_ptr() + 4 * f), 0, sp) == 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            launch_split()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            launch_split()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        same = bool(torch.equal(out.cpu(), ref)) if ref is not None else None
        print(json.dumps({"alloc": "torch, one buffer, launches of %d blocks" % per, "blocks": n, "ms": round(ms, 4),
                          "GiBps": round(n * L / (ms / 1e3) / 2**30, 1),
                          "pct_8TBs": round(100 * n * L / (ms / 1e3) / 8e12, 2), "crcs_equal_torch": same}), flush=True)
    del keep
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    # the same blocks held as ten separate 1M-block allocations, one launch each
    chunks = []
    for c in range((n + (1 << 20) - 1) >> 20):
        m = min(1 << 20, n - (c << 20))
        t = torch.empty(m * L, dtype=torch.uint8, device="cuda")
        assert lb.lsbm_fill_splitmix64_dev(ctypes.c_void_p(t.data_ptr()), m * L, 0x5EED0000 + (c << 20) * (L // 8), sp) == 0
        chunks.append((t, m))
    def launch_all():
        for c, (t, m) in enumerate(chunks):
            assert lb.lsbm_crc32c_fixed_dev(ctypes.c_void_p(t.data_ptr()), L, L, m, None,
                                            ctypes.c_void_p(out.data_ptr() + 4 * (c << 20)), 0, sp) == 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        launch_all()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        launch_all()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    same = bool(torch.equal(out.cpu(), ref)) if ref is not None else None
    print(json.dumps({"alloc": "torch, 1M-block chunks", "blocks": n, "ms": round(ms, 4),
                      "GiBps": round(n * L / (ms / 1e3) / 2**30, 1), "pct_8TBs": round(100 * n * L / (ms / 1e3) / 8e12, 2),
                      "crcs_equal_torch": same}), flush=True)


if __name__ == "__main__":
    main()
