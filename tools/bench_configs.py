#!/usr/bin/env python3
"""Secondary measurements: configs 3 and 4 of BASELINE.json and the
host-staged (PCIe-inclusive) rate.  One JSON line per measurement.

  config3   1M x 64 KiB device-resident blocks (fixed-stride kernel)
  config4   10M blocks, n = min(65536, 512*r + u), r ~ Zipf(0.99) over 1..128,
            u ~ U[0, 511], densely packed at arbitrary alignment (ragged path)
  host      host-staged batches: pinned host buffer -> GPU -> 4 B/block back
  config1   db_bench's CRC mix (BASELINE.json configs[0]): 45,036
            SSTable data blocks of 4117-4122 B + 56 index/filter/meta blocks of
            31-202 KB sealed by lsbm_sst_seal_dev, and 97,597 WAL records of
            0-2540 B (mean 1270) sealed in a log image by lsbm_log_seal_dev;
            beside it the reference's own Extend loop on one host core

Lengths are drawn from splitmix64 streams (seed 0x5EED0002), not the survey's
mt19937_64, so that numpy regenerates them bit for bit; bytes are the on-device
splitmix64 stream (seeds 0x5EED0001 / 0x5EED0003).  Every run spot-checks
sampled blocks against the oracle.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from golden.splitmix import splitmix64, stream_bytes  # noqa: E402

HBM = 8000.0


def zipf_lengths(n, seed=0x5EED0002, ranks=128, theta=0.99):
    """n = min(65536, 512*r + u): r ~ Zipf(theta) on 1..ranks, u ~ U[0, 511]."""
    w = 1.0 / np.arange(1, ranks + 1, dtype=np.float64) ** theta
    cdf = np.cumsum(w) / w.sum()
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        a = splitmix64(np.uint64(seed) + 2 * idx)
        b = splitmix64(np.uint64(seed) + 2 * idx + np.uint64(1))
    u01 = (a >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    r = np.searchsorted(cdf, u01, side="right") + 1
    u = (b % np.uint64(512)).astype(np.int64)
    return np.minimum(65536, 512 * r + u).astype(np.int64)


def time_launches(fn, stream, reps=10, warm=2, spin_s=None):
    """Seconds per launch of fn.  Before the warm-up launches, fn runs for
    spin_s seconds: after host-side pauses the GPU clock has dropped, and a
    few launches are not enough to bring it back."""
    import torch
    if spin_s is None:  # LSBM_SPIN_S=0 under rocprofv3 --pmc (every dispatch is counted)
        spin_s = float(os.environ.get("LSBM_SPIN_S", "0.3"))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < spin_s:
        fn()
        torch.cuda.synchronize()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def oracle():
    from conftest import Oracle
    return Oracle(os.path.join(REPO, "oracle", "liboracle_crc32c.so"))


def config3(args):
    import torch
    from lsbm_amd import engine
    n, L, seed = args.c3_blocks, 65536, 0x5EED0001
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, seed)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_fixed(d, L, L, n, out=out, stream=s), s)
    got = out.cpu().numpy().view(np.uint32)
    o = oracle()
    rng = np.random.default_rng(3)
    bad = sum(int(got[b] != o.value(stream_bytes(seed, int(b) * L, L).tobytes()))
              for b in rng.choice(n, 64, replace=False))
    gbps = n * L / t / 1e9
    print(json.dumps({"config": "config3", "blocks": n, "block_bytes": L, "ms": round(t * 1e3, 3),
                      "GiBps": round(n * L / t / 2**30, 1), "GBps": round(gbps, 1),
                      "pct_hbm_peak": round(100 * gbps / HBM, 2), "sample_mismatches": bad}),
          flush=True)
    del d


def units4k(args):
    """config 2's geometry (1M x 4096 B, stride 4096) through the ragged
    kernel (offsets batch): the ragged path's overhead against the fixed one."""
    import torch
    from lsbm_amd import engine
    n, L, seed = 1 << 20, 4096, 0x5EED0000
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, seed)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_batch(d, offs, out=out, stream=s), s)
    ref = engine.crc32c_fixed(d, L, L, n)
    tf = time_launches(lambda: engine.crc32c_fixed(d, L, L, n, out=ref, stream=s), s)
    gbps, gf = n * L / t / 1e9, n * L / tf / 1e9
    print(json.dumps({"config": "units4k", "blocks": n, "ms": round(t * 1e3, 3), "GBps": round(gbps, 1),
                      "pct_hbm_peak": round(100 * gbps / HBM, 2),
                      "fixed_pct_hbm_peak": round(100 * gf / HBM, 2),
                      "agree_with_fixed": bool(torch.equal(out, ref))}), flush=True)
    del d


def c4uniform(args):
    """config 4's byte count with every block the same length (the mean, 12,534 B):
    what config 4 would run at if the units of a round were equal (lockstep)."""
    import torch
    from lsbm_amd import engine
    n = args.c4_blocks
    lens = np.full(n, 12534, dtype=np.int64)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    offs += 5
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0003)
    do = torch.from_numpy(offs).to("cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_batch(d, do, out=out, stream=s), s, reps=5, warm=1)
    gbps = int(lens.sum()) / t / 1e9
    print(json.dumps({"config": "c4uniform", "blocks": n, "ms": round(t * 1e3, 3),
                      "pct_hbm_peak": round(100 * gbps / HBM, 2)}), flush=True)
    del d, do


def c4sorted(args):
    """(diagnostic) config 4's exact block lengths, sorted (descending): the
    same bytes with every round's 8 units alike -- the lock-step loss."""
    import torch
    from lsbm_amd import engine
    n = args.c4_blocks
    lens = np.sort(zipf_lengths(n))[::-1].copy()
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    offs += 5
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0003)
    do = torch.from_numpy(offs).to("cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_batch(d, do, out=out, stream=s), s, reps=5, warm=1)
    gbps = int(lens.sum()) / t / 1e9
    print(json.dumps({"config": "c4sorted", "blocks": n, "ms": round(t * 1e3, 3),
                      "pct_hbm_peak": round(100 * gbps / HBM, 2)}), flush=True)
    del d, do


def usweep(args):
    """(diagnostic) equal-length blocks through the ragged kernel, 16 GiB per
    length, 5 bytes off alignment: the per-round cost against the unit count."""
    import torch
    from lsbm_amd import engine
    total = args.sweep_gib << 30
    d = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0003)
    s = torch.cuda.current_stream()
    for L in args.sweep_lens:
        n = total // L
        do = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda") + 5
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        t = time_launches(lambda: engine.crc32c_batch(d, do, out=out, stream=s), s, reps=5, warm=1)
        print(json.dumps({"config": "usweep", "len": L, "blocks": n, "ms": round(t * 1e3, 3),
                          "pct_hbm_peak": round(100 * n * L / t / 1e9 / HBM, 2)}), flush=True)
    del d


def config4(args):
    import torch
    from lsbm_amd import engine
    n = args.c4_blocks
    lens = zipf_lengths(n)
    offs = np.zeros(n + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    start_pad = 5  # dense packing at an arbitrary alignment
    offs += start_pad
    total = int(offs[-1]) + 16
    seed = 0x5EED0003
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, seed)
    do = torch.from_numpy(offs).to("cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_batch(d, do, out=out, stream=s), s, reps=5, warm=1)
    got = out.cpu().numpy().view(np.uint32)
    o = oracle()
    rng = np.random.default_rng(4)
    bad = 0
    for b in rng.choice(n, 64, replace=False):
        blk = stream_bytes(seed, int(offs[b]), int(lens[b])).tobytes()
        bad += int(got[b] != o.value(blk))
    payload = int(lens.sum())
    gbps = payload / t / 1e9
    print(json.dumps({"config": "config4", "blocks": n, "payload_GiB": round(payload / 2**30, 2),
                      "mean_len": round(float(lens.mean()), 1),
                      "frac_le_4k": round(float((lens <= 4096).mean()), 3),
                      "ms": round(t * 1e3, 3), "GiBps": round(payload / t / 2**30, 1),
                      "GBps": round(gbps, 1), "pct_hbm_peak": round(100 * gbps / HBM, 2),
                      "sample_mismatches": bad}), flush=True)
    del d, do


def host_staged(args):
    import torch
    from lsbm_amd import engine
    n, L = args.host_blocks, 4096
    # pinned host source (hipHostMalloc via torch), bytes of the config-2 stream
    src = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    src.numpy()[:] = stream_bytes(0x5EED0000, 0, n * L)
    offs = np.arange(0, (n + 1) * L, L, dtype=np.uint64)
    h = src.numpy()
    engine.crc32c_batch_host(h, offs)  # warm: staging buffers, first DMA touch of the pages
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        got = engine.crc32c_batch_host(h, offs)
    t = (time.perf_counter() - t0) / reps
    o = oracle()
    bad = sum(int(got[b] != o.value(h[b * L:(b + 1) * L].tobytes())) for b in range(0, n, n // 64))
    print(json.dumps({"config": "host_staged", "blocks": n, "block_bytes": L,
                      "s": round(t, 4), "GiBps": round(n * L / t / 2**30, 2),
                      "GBps": round(n * L / t / 1e9, 2), "sample_mismatches": bad,
                      "note": "pinned source; includes host gather into staging, H2D, kernel, "
                              "4 B/block D2H"}), flush=True)


def sst4118(args):
    """1M real-size SSTable data blocks (4118 B, the db_bench mode),
    densely packed with their 5-byte trailers, through the ragged kernel:
    block || type CRCs as ReadBlock's verify computes them."""
    import torch
    from lsbm_amd import engine
    n, L = args.sst_blocks, 4118
    offs = (np.arange(n + 1, dtype=np.int64) * (L + 5))
    ext = np.stack([offs[:-1], np.full(n, L + 1, dtype=np.int64)], 1).reshape(-1)
    d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    engine.fill_splitmix64(d, 0x5EED0005)
    de = torch.from_numpy(ext).to("cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    t = time_launches(lambda: engine.crc32c_extents(d, de, out=out, stream=s), s, reps=10)
    got = out.cpu().numpy().view(np.uint32)
    o = oracle()
    rng = np.random.default_rng(6)
    bad = sum(int(got[b] != o.value(stream_bytes(0x5EED0005, int(offs[b]), L + 1).tobytes()))
              for b in rng.choice(n, 64, replace=False))
    gbps = n * (L + 1) / t / 1e9
    # the SSTable entry points on the same image: WriteRawBlock seal, ReadBlock verify
    from lsbm_amd import table
    handles = torch.from_numpy(np.stack([offs[:-1], np.full(n, L, dtype=np.int64)], 1)
                               .reshape(-1).copy()).to("cuda")
    types = torch.zeros(n, dtype=torch.uint8, device="cuda")
    t_seal = time_launches(lambda: table.seal_blocks(d, handles, types, stream=s), s, reps=10)
    t_ver = time_launches(lambda: table.verify_blocks(d, handles, stream=s), s, reps=10)
    tc_out = torch.empty(n, dtype=torch.int32, device="cuda")
    tc_nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    t_tc = time_launches(lambda: table.trailer_crcs(d, handles, types, stream=s, out=tc_out,
                                                    nbad=tc_nbad), s, reps=10)
    img = d.cpu().numpy()
    tc_host = tc_out.cpu().numpy().view(np.uint32)
    ends = offs[:-1] + L
    stored = (img[ends + 1].astype(np.uint32) | (img[ends + 2].astype(np.uint32) << 8) |
              (img[ends + 3].astype(np.uint32) << 16) | (img[ends + 4].astype(np.uint32) << 24))
    g_tc = n * L / t_tc / 1e9
    # the extents timing again, after the others (clock / ordering check)
    t2 = time_launches(lambda: engine.crc32c_extents(d, de, out=out, stream=s), s, reps=10)
    ok, nbad = table.verify_blocks(d, handles, stream=s)
    g_seal, g_ver = n * (L + 1) / t_seal / 1e9, n * (L + 1) / t_ver / 1e9
    print(json.dumps({"config": "sst4118", "blocks": n, "block_bytes": L + 1, "ms": round(t * 1e3, 3),
                      "GBps": round(gbps, 1), "pct_hbm_peak": round(100 * gbps / HBM, 2),
                      "sst_seal": {"ms": round(t_seal * 1e3, 3), "GBps": round(g_seal, 1),
                                   "pct_hbm_peak": round(100 * g_seal / HBM, 2)},
                      "ext_again_pct_hbm_peak": round(100 * n * (L + 1) / t2 / 1e9 / HBM, 2),
                      "sst_trailer_crcs": {"ms": round(t_tc * 1e3, 3), "GBps": round(g_tc, 1),
                                           "pct_hbm_peak": round(100 * g_tc / HBM, 2),
                                           "equal_sealed": bool(np.array_equal(tc_host, stored))},
                      "sst_verify": {"ms": round(t_ver * 1e3, 3), "GBps": round(g_ver, 1),
                                     "pct_hbm_peak": round(100 * g_ver / HBM, 2),
                                     "all_ok": bool(ok.all()) and int(nbad.item()) == 0},
                      "sample_mismatches": bad}), flush=True)


def config1(args):
    import ctypes
    import torch
    from golden.splitmix import printable_bytes
    from lsbm_amd import log, table
    rng = np.random.default_rng(0xC1)
    # 45,036 data blocks (4117 x 12,621, 4118 x 21,072, 4119 x 10,203,
    # 4120 x 1,033, the rest 4121-4122) + 56 index/filter/meta blocks of 31-202 KB
    sizes = np.array([4117] * 12621 + [4118] * 21072 + [4119] * 10203 + [4120] * 1033 +
                     [4121] * 60 + [4122] * 47 + list(rng.integers(31 << 10, 202 << 10, 56)),
                     dtype=np.int64)
    rng.shuffle(sizes)
    handles, total = table.layout_blocks(sizes)
    img = printable_bytes(0xC1, int(total))
    d = torch.from_numpy(img).to("cuda")
    dh = torch.from_numpy(np.ascontiguousarray(handles, dtype=np.int64)).to("cuda")
    types = torch.zeros(sizes.size, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    t_sst = time_launches(lambda: table.seal_blocks(d, dh, types, stream=s), s, reps=10)
    sealed = d.cpu().numpy()
    lens = rng.integers(0, 2541, size=97597)
    pay = printable_bytes(0xC2, int(lens.sum()))
    offs = np.concatenate([[0], np.cumsum(lens)])
    wimg, heads = log.layout_records(pay[offs[i]:offs[i + 1]] for i in range(lens.size))
    dw = torch.from_numpy(wimg).to("cuda")
    dwh = torch.from_numpy(heads).to("cuda")
    t_wal = time_launches(lambda: log.seal_records(dw, dwh, stream=s), s, reps=10)
    wsealed = dw.cpu().numpy()
    sst_bytes = int(sizes.sum()) + sizes.size  # block || type
    # reference Extend loop, one core: block || type (WriteRawBlock) and
    # type_crc_[t] extended over the payload (EmitPhysicalRecord)
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so"))
    ref.ref_batch_extents.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64]
    ext = np.stack([handles[0::2], handles[1::2] + 1], 1).astype(np.uint64).reshape(-1)
    out = np.empty(sizes.size, dtype=np.uint32)
    t0 = time.perf_counter()
    ref.ref_batch_extents(sealed.ctypes.data, ext.ctypes.data, None, out.ctypes.data, sizes.size)
    c_sst = time.perf_counter() - t0
    plen = (wsealed[heads + 4].astype(np.uint64) | (wsealed[heads + 5].astype(np.uint64) << 8))
    wext = np.stack([heads.astype(np.uint64) + 6, plen + 1], 1).reshape(-1)
    wout = np.empty(heads.size, dtype=np.uint32)
    t0 = time.perf_counter()
    ref.ref_batch_extents(wsealed.ctypes.data, wext.ctypes.data, None, wout.ctypes.data, heads.size)
    c_wal = time.perf_counter() - t0
    o = oracle()
    # the GPU's trailers / headers are what the reference computes
    bad = sum(int(o.mask(int(out[i])) != int.from_bytes(sealed[handles[2 * i] + sizes[i] + 1:
                                                               handles[2 * i] + sizes[i] + 5].tobytes(),
                                                        "little"))
              for i in range(0, sizes.size, 97))
    bad += sum(int(o.mask(int(wout[i])) != int.from_bytes(wsealed[heads[i]:heads[i] + 4].tobytes(), "little"))
               for i in range(0, heads.size, 97))
    crc_bytes = sst_bytes + int(plen.sum()) + heads.size
    print(json.dumps({"config": "config1", "sst_blocks": int(sizes.size), "sst_crc_bytes": sst_bytes,
                      "wal_records": int(lens.size), "wal_physical": int(heads.size),
                      "wal_crc_bytes": int(plen.sum()) + int(heads.size),
                      "gpu_ms": {"sst_seal": round(t_sst * 1e3, 3), "log_seal": round(t_wal * 1e3, 3)},
                      "gpu_GBps": round(crc_bytes / (t_sst + t_wal) / 1e9, 1),
                      "cpu_reference_1core": {"s": round(c_sst + c_wal, 4),
                                              "GBps": round(crc_bytes / (c_sst + c_wal) / 1e9, 3)},
                      "speedup_vs_1core": round((c_sst + c_wal) / (t_sst + t_wal), 1),
                      "sample_mismatches": bad,
                      "note": "device-resident images; the reference run writes these through "
                              "fwrite on one thread (SURVEY.md 3.5)"}), flush=True)


def wal(args):
    """A WAL group commit on the device: 400K db_bench-sized records (0-2540 B,
    ~0.5 GB framed), every header sealed (lsbm_log_seal_dev, with and without
    the dense CRC output), the dense CRCs alone (lsbm_log_crcs_dev) and the
    recovery check (lsbm_log_verify_dev).  Bytes = type + payload per header."""
    import ctypes
    import torch
    from golden.splitmix import printable_bytes
    from lsbm_amd import log
    from lsbm_amd._lib import lib
    rng = np.random.default_rng(0xA1)
    lens = rng.integers(0, 2541, size=args.wal_records)
    if args.wal_fixed_len is not None:  # (diagnostic: no length spread)
        lens[:] = args.wal_fixed_len
    pay = printable_bytes(0xA2, int(lens.sum()))
    offs = np.concatenate([[0], np.cumsum(lens)])
    wimg, heads = log.layout_records(pay[offs[i]:offs[i + 1]] for i in range(lens.size))
    d = torch.from_numpy(wimg).to("cuda")
    dh = torch.from_numpy(heads).to("cuda")
    n = heads.size
    masked = torch.empty(n, dtype=torch.int32, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    L = lib()
    dp, hp, mp, bp, op = (ctypes.c_void_p(t.data_ptr()) for t in (d, dh, masked, nbad, ok))
    nb = ctypes.c_uint64(d.numel())
    t_seal = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp), s)
    t_seal_nm = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hp, n, None, bp, sp), s)
    t_crcs = time_launches(lambda: L.lsbm_log_crcs_dev(dp, nb, hp, n, mp, bp, sp), s)
    nbad.zero_()
    t_ver = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hp, n, op, bp, sp), s)
    torch.cuda.synchronize()
    img = d.cpu().numpy()
    plen = img[heads + 4].astype(np.int64) | (img[heads + 5].astype(np.int64) << 8)
    # (diagnostic) the same bytes as {offset, length} extents: no header load
    ext = torch.from_numpy(np.stack([heads.astype(np.int64) + 6, plen + 1], 1).reshape(-1)).to("cuda")
    ep = ctypes.c_void_p(ext.data_ptr())
    t_ext = time_launches(lambda: L.lsbm_crc32c_extents_dev(dp, ep, n, None, mp, 0, sp), s)
    crc_bytes = int(plen.sum()) + n
    # (diagnostic) the same headers passed length-sorted within windows of 512
    # (the kernel takes header offsets in any order): a round's 8 records alike
    W = 512
    perm = np.concatenate([i + np.argsort(plen[i:i + W], kind="stable") for i in range(0, n, W)])
    dhs = torch.from_numpy(heads[perm].astype(heads.dtype)).to("cuda")
    hsp = ctypes.c_void_p(dhs.data_ptr())
    t_seal_sorted = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hsp, n, mp, bp, sp), s)
    nbad.zero_()
    t_ver_sorted = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hsp, n, op, bp, sp), s)
    sorted_ok = bool(ok.all().item())
    # every header offset shuffled (no order at all), and both out-of-order
    # inputs on the units kernel alone (lsbm_test_ragged_kernel(1)) in the same run
    dhx = torch.from_numpy(heads[np.random.default_rng(0xA3).permutation(n)].astype(heads.dtype)).to("cuda")
    hxp = ctypes.c_void_p(dhx.data_ptr())
    t_seal_shuf = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hxp, n, mp, bp, sp), s)
    t_ver_shuf = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hxp, n, op, bp, sp), s)
    shuf_ok = bool(ok.all().item())
    L.lsbm_test_ragged_kernel(1)
    try:
        u_seal_sorted = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hsp, n, mp, bp, sp), s)
        u_ver_sorted = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hsp, n, op, bp, sp), s)
        u_seal_shuf = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hxp, n, mp, bp, sp), s)
        u_ver_shuf = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hxp, n, op, bp, sp), s)
        u_seal = time_launches(lambda: L.lsbm_log_seal_dev(dp, nb, hp, n, mp, bp, sp), s)
        u_ver = time_launches(lambda: L.lsbm_log_verify_dev(dp, nb, hp, n, op, bp, sp), s)
        # (diagnostic) the stream kernel over the same bytes as {offset, length}
        # extents: no record-length loads at all (the bound for deriving lengths)
        L.lsbm_test_ragged_kernel(2)
        t_ext_stream = time_launches(lambda: L.lsbm_crc32c_extents_dev(dp, ep, n, None, mp, 0, sp), s)
    finally:
        L.lsbm_test_ragged_kernel(0)
    o = oracle()
    bad = 0
    for i in range(0, n, max(1, n // 2000)):
        h = int(heads[i])
        want = o.mask(o.value(img[h + 6:h + 7 + int(plen[i])].tobytes()))
        bad += int(want != int.from_bytes(img[h:h + 4].tobytes(), "little"))
    pct = lambda t: round(crc_bytes / t / 1e9 / HBM * 100, 2)
    print(json.dumps({"config": "wal", "fixed_len": args.wal_fixed_len, "records": int(lens.size), "physical": int(n), "crc_bytes": crc_bytes,
                      "log_seal": {"ms": round(t_seal * 1e3, 3), "pct_hbm_peak": pct(t_seal)},
                      "log_seal_no_out": {"ms": round(t_seal_nm * 1e3, 3), "pct_hbm_peak": pct(t_seal_nm)},
                      "log_crcs": {"ms": round(t_crcs * 1e3, 3), "pct_hbm_peak": pct(t_crcs)},
                      "log_verify": {"ms": round(t_ver * 1e3, 3), "pct_hbm_peak": pct(t_ver),
                                     "all_ok": bool(ok.all().item())},
                      "extents_same_bytes": {"ms": round(t_ext * 1e3, 3), "pct_hbm_peak": pct(t_ext),
                                             "stream_kernel_pct_hbm_peak": pct(t_ext_stream)},
                      "len_sorted_512": {"seal_pct_hbm_peak": pct(t_seal_sorted), "verify_pct_hbm_peak": pct(t_ver_sorted),
                                         "verify_all_ok": sorted_ok},
                      "shuffled": {"seal_pct_hbm_peak": pct(t_seal_shuf), "verify_pct_hbm_peak": pct(t_ver_shuf),
                                   "verify_all_ok": shuf_ok},
                      "units_kernel": {"in_order": {"seal": pct(u_seal), "verify": pct(u_ver)},
                                       "len_sorted_512": {"seal": pct(u_seal_sorted), "verify": pct(u_ver_sorted)},
                                       "shuffled": {"seal": pct(u_seal_shuf), "verify": pct(u_ver_shuf)}},
                      "sample_mismatches": bad}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", nargs="*", default=["config1", "config3", "config4", "host"])
    p.add_argument("--c3-blocks", type=int, default=1 << 20)
    p.add_argument("--c4-blocks", type=int, default=10_000_000)
    p.add_argument("--host-blocks", type=int, default=1 << 18)
    p.add_argument("--sst-blocks", type=int, default=1 << 20)
    p.add_argument("--wal-records", type=int, default=400_000)
    p.add_argument("--wal-fixed-len", type=int, default=None)
    p.add_argument("--sweep-gib", type=int, default=16)
    p.add_argument("--sweep-lens", type=int, nargs="+",
                   default=[1024, 2048, 4096, 6144, 8192, 12288, 16384, 24576, 49152, 65536])
    args = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from lsbm_amd import engine
    engine.init(0)
    for w in args.which:
        {"sst4118": sst4118, "units4k": units4k, "c4uniform": c4uniform, "c4sorted": c4sorted, "usweep": usweep, "config1": config1, "config3": config3, "config4": config4, "host": host_staged,
         "wal": wal}[w](args)


if __name__ == "__main__":
    main()
