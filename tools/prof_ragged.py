#!/usr/bin/env python3
"""Profiling driver for the ragged CRC kernels (run under rocprofv3 on the GPU
box): a few launches of one device-resident workload, no clock spin-up (every
dispatch is profiled).

  wal       400K WAL records (0-2540 B) in a framed log image: lsbm_log_verify_dev
  walseal   the same image: lsbm_log_seal_dev
  units4k   1M x 4 KiB blocks as an offsets[] batch: lsbm_crc32c_batch_dev
  sst       1M x 4,118-B blocks with trailers: lsbm_sst_verify_dev
  c4        2M blocks of config 4's Zipf lengths (23 GiB): lsbm_crc32c_batch_dev

LSBM_RAGGED_KERNEL=units | stream selects the kernel (lsbm_amd/csrc/crc32c_kernels.hip
ragged_uses_stream; by default offsets[] batches take the stream kernel).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, HERE)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which")
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--stats", action="store_true",
                   help="print the stream kernel's event counters (tools/stream_stats.sh build)")
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from lsbm_amd import engine, log, table
    from lsbm_amd._lib import lib
    from golden.splitmix import printable_bytes
    engine.init(0)
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    L = lib()
    if a.which in ("wal", "walseal"):
        rng = np.random.default_rng(0xA1)
        lens = rng.integers(0, 2541, size=400_000)
        pay = printable_bytes(0xA2, int(lens.sum()))
        offs = np.concatenate([[0], np.cumsum(lens)])
        wimg, heads = log.layout_records(pay[offs[i]:offs[i + 1]] for i in range(lens.size))
        d = torch.from_numpy(wimg).to("cuda")
        dh = torch.from_numpy(heads).to("cuda")
        n = heads.size
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")
        nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
        masked = torch.empty(n, dtype=torch.int32, device="cuda")
        dp, hp, op, bp, mp = (ctypes.c_void_p(t.data_ptr()) for t in (d, dh, ok, nbad, masked))
        nb = ctypes.c_uint64(d.numel())
        L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp)
        if a.which == "wal":
            fn = lambda: L.lsbm_log_verify_dev(dp, nb, hp, n, op, bp, sp)
        else:
            fn = lambda: L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp)
    elif a.which == "units4k":
        n, ln = 1 << 20, 4096
        d = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0000)
        offs = torch.arange(0, (n + 1) * ln, ln, dtype=torch.int64, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        fn = lambda: engine.crc32c_batch(d, offs, out=out, stream=s)
    elif a.which in ("sst", "sstseal"):
        n, ln = 1 << 20, 4118
        offs = np.arange(n + 1, dtype=np.int64) * (ln + 5)
        d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0005)
        handles = torch.from_numpy(np.stack([offs[:-1], np.full(n, ln, dtype=np.int64)], 1)
                                   .reshape(-1).copy()).to("cuda")
        types = torch.zeros(n, dtype=torch.uint8, device="cuda")
        table.seal_blocks(d, handles, types, stream=s)
        if a.which == "sst":
            fn = lambda: table.verify_blocks(d, handles, stream=s)
        else:  # lsbm_sst_seal_dev: dense CRCs + per-wave trailer merges
            fn = lambda: table.seal_blocks(d, handles, types, stream=s)
    elif a.which == "c4":
        from bench_configs import zipf_lengths
        n = 2_000_000
        lens = zipf_lengths(n)
        offs = np.zeros(n + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        offs += 5
        d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0003)
        do = torch.from_numpy(offs).to("cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        fn = lambda: engine.crc32c_batch(d, do, out=out, stream=s)
    else:
        raise SystemExit("unknown workload " + a.which)
    if a.stats:
        fn()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        L.lsbm_stream_stats(buf)  # clear
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    if a.stats:
        assert L.lsbm_stream_stats(buf) == 0
        names = ["wave_rows", "slow_rows", "gen_halves", "gen_iters", "flushes", "merges",
                 "subpieces", "group_events"]
        st = {k: buf[i] / a.reps for i, k in enumerate(names)}
        kib = d.numel() / 1024.0
        print(a.which, " ".join(f"{k}={v:.0f}" for k, v in st.items()))
        print(a.which, "per KiB:", " ".join(f"{k}={v / kib:.3f}" for k, v in st.items()))
        tn = ["setup", "loop", "flush", "general", "unused", "tail", "finish(tail)"]
        tt = [buf[8 + i] / a.reps for i in range(len(tn))]
        tot = tt[0] + tt[1] + tt[5]
        print(a.which, "wave cycles %.3g:" % tot, " ".join(f"{k}={v / tot:.3f}" for k, v in zip(tn, tt)))


if __name__ == "__main__":
    main()
