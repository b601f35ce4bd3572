#!/usr/bin/env python3
"""One device entry point per process, for rocprofv3 (tools/roofline.sh).

    python tools/roofline_all.py ENTRY

ENTRY is one of the workloads below; the process sets it up, runs it for a
0.3 s clock spin-up (LSBM_SPIN_S) plus warm-up and timed launches, checks
sampled results against the oracle, and prints ONE JSON line naming the
entry, its kernel (a regex over rocprof kernel names) and its ALGORITHMIC
bytes per launch.  Run under `rocprofv3 --kernel-trace --stats`, the kernel's
average duration comes from rocprof itself, not from HIP events; under a
`--pmc FETCH_SIZE` pass, its HBM bytes.  tools/roofline_summary.py joins
the three.

  fixed4k     config 2: 1M x 4096 B, lsbm_crc32c_fixed_dev        (block bytes)
  config3     1M x 64 KiB, lsbm_crc32c_fixed_dev                   (block bytes)
  config4     10M Zipf blocks, 117 GiB, lsbm_crc32c_batch_dev      (block bytes)
  sst_ext     1M x 4,118-B SSTable blocks, block || type as extents (n (L+1))
  sst_seal    the same image, lsbm_sst_seal_dev                    (n (L+1))
  sst_crcs    lsbm_sst_trailer_crcs_dev                            (n (L+1))
  sst_verify  lsbm_sst_verify_dev                                  (n (L+1))
  log_seal    400K db_bench-sized WAL records, lsbm_log_seal_dev   (type || payload)
  log_crcs    lsbm_log_crcs_dev                                    (type || payload)
  log_verify  lsbm_log_verify_dev                                  (type || payload)
(The SSTable entries count the type byte: every one of them CRCs block || type.)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))

from bench_configs import oracle, time_launches, zipf_lengths  # noqa: E402
from golden.splitmix import stream_bytes  # noqa: E402


def line(entry, kernel, alg, t, bad, **kw):
    d = {"entry": entry, "kernel_regex": kernel, "algorithmic_bytes": int(alg), "events_ms": round(t * 1e3, 4),
         "events_pct_hbm": round(100 * alg / t / 8e12, 2), "sample_mismatches": int(bad)}
    d.update(kw)
    print(json.dumps(d), flush=True)


def fixed(entry, L, n, seed, reps):
    import torch
    from lsbm_amd import engine
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, seed)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_fixed(d, L, L, n, out=out, stream=s), s, reps=reps)
    got = out.cpu().numpy().view(np.uint32)
    o = oracle()
    bad = sum(int(got[b] != o.value(stream_bytes(seed, int(b) * L, L).tobytes()))
              for b in np.random.default_rng(1).choice(n, 32, replace=False))
    line(entry, rf"crc32c_fixed_kernel<false, {512 if L == 65536 else 32}u>", n * L, t, bad,
         blocks=n, block_bytes=L)


def config4(reps):
    import torch
    from lsbm_amd import engine
    n = 10_000_000
    lens = zipf_lengths(n)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    offs += 5
    seed = 0x5EED0003
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, seed)
    do = torch.from_numpy(offs).to("cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_batch(d, do, out=out, stream=s), s, reps=reps, warm=1)
    got = out.cpu().numpy().view(np.uint32)
    o = oracle()
    bad = sum(int(got[b] != o.value(stream_bytes(seed, int(offs[b]), int(lens[b])).tobytes()))
              for b in np.random.default_rng(4).choice(n, 32, replace=False))
    # the batch's kernels: the chunked sweep's bounds pre-pass and the stream kernel
    line("config4", r"crc32c_stream_kernel<32u, 0u, 0u>|range_bounds_kernel", int(lens.sum()), t, bad,
         blocks=n, mean_len=round(float(lens.mean()), 1))


def sst(entry, reps):
    import torch
    from lsbm_amd import engine, table
    n, L = 1 << 20, 4118
    offs = np.arange(n + 1, dtype=np.int64) * (L + 5)
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0005)
    handles = torch.from_numpy(np.stack([offs[:-1], np.full(n, L, dtype=np.int64)], 1).reshape(-1).copy()).to("cuda")
    types = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    o = oracle()
    sample = np.random.default_rng(6).choice(n, 32, replace=False)
    if entry == "sst_ext":
        ext = torch.from_numpy(np.stack([offs[:-1], np.full(n, L + 1, dtype=np.int64)], 1).reshape(-1)).to("cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        t = time_launches(lambda: engine.crc32c_extents(d, ext, out=out, stream=s), s, reps=reps)
        got = out.cpu().numpy().view(np.uint32)
        bad = sum(int(got[b] != o.value(stream_bytes(0x5EED0005, int(offs[b]), L + 1).tobytes())) for b in sample)
        return line(entry, r"crc32c_units_kernel<48u, 0u, 1u, ", n * (L + 1), t, bad, blocks=n)
    # seal first (the other entries read its trailers), untimed when it is not the entry
    if entry == "sst_seal":
        t = time_launches(lambda: table.seal_blocks(d, handles, types, stream=s), s, reps=reps)
    else:
        table.seal_blocks(d, handles, types, stream=s)
        torch.cuda.synchronize()
    img = d.cpu().numpy()
    ends = offs[:-1] + L
    stored = (img[ends + 1].astype(np.uint32) | (img[ends + 2].astype(np.uint32) << 8) |
              (img[ends + 3].astype(np.uint32) << 16) | (img[ends + 4].astype(np.uint32) << 24))
    bad = sum(int(stored[b] != o.mask(o.value(img[offs[b]:offs[b] + L + 1].tobytes()))) for b in sample)
    if entry == "sst_seal":
        return line(entry, r"crc32c_units_kernel<40u, 6u, 1u, ", n * (L + 1), t, bad, blocks=n)
    if entry == "sst_crcs":
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        nb = torch.zeros(1, dtype=torch.int32, device="cuda")
        t = time_launches(lambda: table.trailer_crcs(d, handles, types, stream=s, out=out, nbad=nb), s, reps=reps)
        bad += int(not np.array_equal(out.cpu().numpy().view(np.uint32), stored))
        return line(entry, r"crc32c_units_kernel<40u, 6u, 1u, ", n * (L + 1), t, bad, blocks=n)
    if entry == "sst_verify":
        t = time_launches(lambda: table.verify_blocks(d, handles, stream=s), s, reps=reps)
        ok, nbad = table.verify_blocks(d, handles, stream=s)
        bad += int(not bool(ok.all().item()) or int(nbad.item()) != 0)
        return line(entry, r"crc32c_units_kernel<40u, 3u, 1u, ", n * (L + 1), t, bad, blocks=n)
    raise SystemExit(f"unknown entry {entry}")


def wal(entry, reps):
    import torch
    from golden.splitmix import printable_bytes
    from lsbm_amd import log
    from lsbm_amd._lib import lib
    rng = np.random.default_rng(0xA1)
    lens = rng.integers(0, 2541, size=400_000)
    pay = printable_bytes(0xA2, int(lens.sum()))
    po = np.concatenate([[0], np.cumsum(lens)])
    wimg, heads = log.layout_records(pay[po[i]:po[i + 1]] for i in range(lens.size))
    d = torch.from_numpy(wimg).to("cuda")
    dh = torch.from_numpy(heads).to("cuda")
    n = heads.size
    masked = torch.empty(n, dtype=torch.int32, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    L = lib()
    dp, hp, mp, bp, op = (ctypes.c_void_p(x.data_ptr()) for x in (d, dh, masked, nbad, ok))
    nb = ctypes.c_uint64(d.numel())
    fn = {"log_seal": lambda: L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp),
          "log_crcs": lambda: L.lsbm_log_crcs_dev(dp, nb, hp, n, mp, bp, sp),
          "log_verify": lambda: L.lsbm_log_verify_dev(dp, nb, hp, n, op, bp, sp)}[entry]
    if entry == "log_verify":
        L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp)
        nbad.zero_()
    t = time_launches(fn, s, reps=reps)
    torch.cuda.synchronize()
    img = d.cpu().numpy()
    plen = img[heads + 4].astype(np.int64) | (img[heads + 5].astype(np.int64) << 8)
    o = oracle()
    bad = 0
    mh = masked.cpu().numpy().view(np.uint32)
    for i in np.random.default_rng(7).choice(n, 32, replace=False):
        h = int(heads[i])
        want = o.mask(o.value(img[h + 6:h + 7 + int(plen[i])].tobytes()))
        # (the dense CRCs leave the image alone: their masked[] is the result)
        got = int(mh[i]) if entry == "log_crcs" else int.from_bytes(img[h:h + 4].tobytes(), "little")
        bad += int(want != got)
    if entry == "log_verify":
        bad += int(not bool(ok.all().item()))
    mode = {"log_seal": 4, "log_crcs": 4, "log_verify": 5}[entry]  # (the dense CRCs: the seal mode without the image)
    line(entry, rf"crc32c_stream_kernel<16u, {mode}u, 3u>", int(plen.sum()) + n, t, bad, records=int(n))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("entry")
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from lsbm_amd import engine
    engine.init(0)
    e = a.entry
    if e == "fixed4k":
        fixed(e, 4096, 1 << 20, 0x5EED0000, a.reps)
    elif e == "config3":
        fixed(e, 65536, 1 << 20, 0x5EED0001, max(3, a.reps // 4))
    elif e == "config4":
        config4(max(3, a.reps // 4))
    elif e.startswith("sst_"):
        sst(e, a.reps)
    elif e.startswith("log_"):
        wal(e, a.reps)
    else:
        raise SystemExit(f"unknown entry {e}")


if __name__ == "__main__":
    main()
