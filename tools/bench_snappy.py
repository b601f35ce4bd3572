#!/usr/bin/env python3
"""Snappy block codec rates on one GPU, db_bench shaped:
~4,118-B data blocks as db_bench's fill workload writes them (BlockBuilder
layout, internal keys "user%019d", 100-byte values that compress to ~50%;
tools/dbbench_blocks.c, the layout of tests/golden/snappy_inputs.py
dbbench_block).  Every block of the batch is distinct (262,144 blocks, 1.08 GB
by default), built on the host and copied to HBM before timing.  One JSON line
per measurement:

  snappy_compress    lsbm_snappy_compress_dev over the batch (WriteBlock's
                     RawCompress, table/table_builder.cc:186)
  snappy_uncompress  lsbm_snappy_uncompress_dev over the compressed batch
                     (ReadBlock's RawUncompress, table/format.cc:130)

value = uncompressed GB/s (raw bytes / kernel time).  The roofline uses the
algorithmic HBM bytes per block: raw + compressed (read one, write the other).
cpu_baseline: libsnappy itself (the pyarrow build the oracle is pinned to) on
every usable host core (one process per core, each over its own share of the
same blocks, started together), with the one-core rate beside it, plus the
oracle's C restatement on one core.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

HBM = 8000.0  # GB/s, MI355X spec


def timed(torch, fn, reps, warm=2, spin_s=None):
    """Seconds per call, after spin_s seconds of untimed calls (the GPU clock
    drops during host-side pauses).  LSBM_SPIN_S=0 under
    rocprofv3 --pmc."""
    if spin_s is None:
        spin_s = float(os.environ.get("LSBM_SPIN_S", "0.3"))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < spin_s:
        fn()
        torch.cuda.synchronize()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def make_blocks(n, seed=7):
    """n distinct db_bench-shaped blocks: (bytes as np.uint8, offsets[n+1])."""
    import subprocess
    so = os.path.join(REPO, "build", "libdbgen.so")
    if not os.path.exists(so):
        os.makedirs(os.path.dirname(so), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", so,
                        os.path.join(HERE, "dbbench_blocks.c")], check=True)
    lib = ctypes.CDLL(so)
    lib.dbgen_blocks.restype = ctypes.c_size_t
    lib.dbgen_blocks.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_void_p]
    need = lib.dbgen_blocks(seed, n, None, 0, None)
    buf = np.empty(need, np.uint8)
    offs = np.empty(n + 1, np.uint64)
    lib.dbgen_blocks(seed, n, buf.ctypes.data, need, offs.ctypes.data)
    return buf, offs


def usable_cores():
    sys.path.insert(0, REPO)
    from bench import usable_cores as uc
    return uc()[0]


_BLOCKS = None  # (buf, offs, compressed list) shared with forked workers


def _worker(args):
    """One process: libsnappy over blocks [lo, hi) for ~seconds; raw bytes/s."""
    kind, lo, hi, seconds, barrier = args
    import pyarrow as pa
    codec = pa.Codec("snappy")
    buf, offs, comp = _BLOCKS
    blocks = [buf[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(lo, hi)]
    raw = sum(len(b) for b in blocks)
    barrier.wait()
    t0, passes = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        if kind == "compress":
            for b in blocks:
                codec.compress(b, asbytes=True)
        else:
            for c, b in zip(comp[lo:hi], blocks):
                codec.decompress(c, decompressed_size=len(b), asbytes=True)
        passes += 1
    return raw * passes, time.perf_counter() - t0


def cpu_baselines(buf, offs, n_sample, seconds=4.0):
    """libsnappy (pyarrow) compress / uncompress over the first n_sample
    blocks: one core, and all usable cores (one forked process per core, each
    over its own share of the sample, started together).  Raw GB/s."""
    global _BLOCKS
    import multiprocessing as mp
    out = {}
    try:
        import pyarrow as pa
    except ImportError:
        return out
    codec = pa.Codec("snappy")
    comp = [codec.compress(buf[int(offs[i]):int(offs[i + 1])].tobytes(), asbytes=True)
            for i in range(n_sample)]
    _BLOCKS = (buf, offs, comp)
    cores = usable_cores()
    ctx = mp.get_context("fork")
    for kind in ("compress", "uncompress"):
        for nproc in (1, cores):
            with ctx.Manager() as m:
                bar = m.Barrier(nproc)
                cut = [n_sample * k // nproc for k in range(nproc + 1)]
                with ctx.Pool(nproc) as pool:
                    res = pool.map(_worker, [(kind, cut[k], cut[k + 1], seconds, bar)
                                             for k in range(nproc)])
            rate = sum(b for b, _ in res) / max(t for _, t in res) / 1e9
            out[f"libsnappy_{kind}_{'1core' if nproc == 1 else 'all'}"] = rate
    out["cores"] = cores
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_snappy.so"))
    m = min(n_sample, 2048)
    data = np.ascontiguousarray(buf[:int(offs[m])])
    o = np.ascontiguousarray(offs[:m + 1])
    lens = np.diff(o)
    caps = (32 + lens + lens // 6).astype(np.uint64)
    oo = np.zeros(m + 1, np.uint64)
    oo[1:] = np.cumsum(caps)
    cout = np.zeros(int(oo[-1]), np.uint8)
    osz = np.zeros(m, np.uint64)
    t0, passes = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds / 2:
        lib.so_compress_batch(ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(o.ctypes.data),
                              ctypes.c_uint64(m), ctypes.c_void_p(cout.ctypes.data),
                              ctypes.c_void_p(oo.ctypes.data), ctypes.c_void_p(osz.ctypes.data))
        passes += 1
    out["oracle_compress"] = data.size * passes / (time.perf_counter() - t0) / 1e9
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--cpu-sample", type=int, default=65536)
    ap.add_argument("--merge", type=int, default=1,
                    help="(diagnostic) concatenate this many consecutive blocks into one: larger blocks")
    args = ap.parse_args()

    buf, offs_h = make_blocks(args.blocks)
    if args.merge > 1:
        offs_h = np.ascontiguousarray(np.concatenate([offs_h[:-1:args.merge], offs_h[-1:]]))
    n = offs_h.size - 1
    # the CPU baseline first, in forked worker processes, before this process
    # touches the GPU (no child ever holds a device context)
    # (--cpu-seconds 0: no CPU baseline, e.g. under rocprofv3 --pmc, whose
    # library has initialised the GPU before this process could fork)
    cpu = cpu_baselines(buf, offs_h, min(n, args.cpu_sample), args.cpu_seconds) if args.cpu_seconds > 0 else {}
    import torch
    from lsbm_amd import engine, snappy
    engine.init(0)
    data = torch.from_numpy(buf).cuda()
    offs = torch.from_numpy(offs_h.astype(np.int64)).cuda()
    raw_bytes = int(offs_h[-1])

    out, oo, ol = snappy.compress(data, offs)
    t_c = timed(torch, lambda: snappy.compress(data, offs, out=out, out_offsets=oo, out_len=ol), args.reps)
    comp_bytes = int(ol.sum().item())
    # sample parity against the oracle
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import SnappyOracle
    orc = SnappyOracle(os.path.join(REPO, "oracle", "liboracle_snappy.so"))
    oo_h, ol_h, out_h = oo.cpu().numpy(), ol.cpu().numpy(), None
    mism = 0
    for i in range(0, n, max(1, n // 512)):
        b = buf[int(offs_h[i]):int(offs_h[i + 1])].tobytes()
        s = int(oo_h[i])
        g = out[s:s + int(ol_h[i])].cpu().numpy().tobytes()
        mism += g != orc.compress(b)

    # pack compressed blocks densely for the decoder
    coffs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(ol, 0, out=coffs[1:])
    idx = torch.repeat_interleave(oo[:-1] - coffs[:-1], ol) + torch.arange(comp_bytes, device="cuda")
    cdata = out[idx]
    uo = offs.clone()
    uout = torch.empty(raw_bytes, dtype=torch.uint8, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    snappy.uncompress(cdata, coffs, out=uout, out_offsets=uo, ok=ok, n_bad=nbad)
    torch.cuda.synchronize()
    rt_ok = bool(torch.equal(uout, data)) and int(nbad.item()) == 0
    nbad.zero_()
    t_u = timed(torch, lambda: snappy.uncompress(cdata, coffs, out=uout, out_offsets=uo, ok=ok,
                                                 n_bad=nbad), args.reps)

    alg = raw_bytes + comp_bytes
    common = {"unit": "GB/s", "higher_is_better": True, "n_gpus": 1, "dtype": "u8",
              "data": "synthetic db_bench-shaped data blocks, %d distinct, resident in HBM" % n,
              "config": {"workload": "%d x ~%d B SSTable data blocks" % (n, raw_bytes // n),
                         "blocks": n, "raw_bytes": raw_bytes, "compressed_bytes": comp_bytes,
                         "ratio": round(comp_bytes / raw_bytes, 4)}}
    for name, t, base in (("snappy_compress", t_c, "libsnappy_compress"),
                          ("snappy_uncompress", t_u, "libsnappy_uncompress")):
        line = dict(metric=name + " raw GB/s", value=round(raw_bytes / t / 1e9, 2), ms=round(t * 1e3, 3),
                    **common)
        line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM, "unit": "GB/s",
                            "frac": round(alg / t / 1e9 / HBM, 4), "traffic": None,
                            "note": "algorithmic bytes = raw + compressed per block; the kernels are "
                                    "latency bound (serial tag walk), see DESIGN.md section 11"}
        if base + "_all" in cpu:
            line["cpu_baseline"] = {"value": round(cpu[base + "_all"], 3), "unit": "GB/s",
                                    "cores": cpu["cores"],
                                    "kind": "libsnappy (pyarrow %s build, the library the oracle is pinned to)"
                                            % __import__("pyarrow").__version__,
                                    "sample": "%d distinct blocks, one process per usable core, ~%.0f s"
                                              % (min(n, args.cpu_sample), args.cpu_seconds),
                                    "single_core": round(cpu[base + "_1core"], 3)}
            line["vs_cpu_all_cores"] = round(raw_bytes / t / 1e9 / cpu[base + "_all"], 2)
        if name == "snappy_compress":
            line["sample_mismatches"] = int(mism)
            line["oracle_compress_1core_GBps"] = round(cpu.get("oracle_compress", 0), 3)
        else:
            line["roundtrip_ok"] = rt_ok
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
