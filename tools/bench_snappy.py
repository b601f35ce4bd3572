#!/usr/bin/env python3
"""Snappy block codec rates on one GPU, db_bench shaped:
~4,118-B data blocks as db_bench's fill workload writes them
(tests/golden/snappy_inputs.py dbbench_block: BlockBuilder layout, internal
keys "user%019d", 100-byte values that compress to ~50%).  A pool of distinct
blocks is built on the host, copied to HBM and tiled to the batch size, so
every block of the batch sits at its own address; all input is resident in
HBM before timing.  One JSON line per measurement:

  snappy_compress    lsbm_snappy_compress_dev over the batch (WriteBlock's
                     RawCompress, table/table_builder.cc:186)
  snappy_uncompress  lsbm_snappy_uncompress_dev over the compressed batch
                     (ReadBlock's RawUncompress, table/format.cc:130)

value = uncompressed GB/s (raw bytes / kernel time).  The roofline uses the
algorithmic HBM bytes per block: raw + compressed (read one, write the other).
cpu_baseline: libsnappy itself (the pyarrow build the oracle is pinned to) on
one host core over a bounded sample, plus the oracle's C restatement.
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


def timed(torch, fn, reps, warm=2):
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


def pool_blocks(n_pool):
    from snappy_inputs import dbbench_block
    blocks, k = [], 0
    for i in range(n_pool):
        b, k = dbbench_block(900000 + i, k)
        blocks.append(b)
    return blocks


def cpu_baselines(blocks, seconds=10.0):
    """(libsnappy compress, libsnappy uncompress, oracle compress) in raw GB/s
    on one core, each over repeated passes of `blocks` for ~seconds/3."""
    out = {}
    try:
        import pyarrow as pa
        codec = pa.Codec("snappy")
        comp = [codec.compress(b, asbytes=True) for b in blocks]
        raw = sum(len(b) for b in blocks)
        for name, fn in (("compress", lambda: [codec.compress(b, asbytes=True) for b in blocks]),
                         ("uncompress", lambda: [codec.decompress(c, decompressed_size=len(b), asbytes=True)
                                                 for c, b in zip(comp, blocks)])):
            t0, passes = time.perf_counter(), 0
            while time.perf_counter() - t0 < seconds / 3:
                fn()
                passes += 1
            out["libsnappy_" + name] = raw * passes / (time.perf_counter() - t0) / 1e9
    except ImportError:
        pass
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_snappy.so"))
    data = np.frombuffer(b"".join(blocks), np.uint8)
    offs = np.zeros(len(blocks) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in blocks])
    caps = np.array([32 + len(b) + len(b) // 6 for b in blocks], np.uint64)
    oo = np.zeros(len(blocks) + 1, np.uint64)
    oo[1:] = np.cumsum(caps)
    cout = np.zeros(int(oo[-1]), np.uint8)
    osz = np.zeros(len(blocks), np.uint64)
    t0, passes = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds / 3:
        lib.so_compress_batch(ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                              ctypes.c_uint64(len(blocks)), ctypes.c_void_p(cout.ctypes.data),
                              ctypes.c_void_p(oo.ctypes.data), ctypes.c_void_p(osz.ctypes.data))
        passes += 1
    out["oracle_compress"] = data.size * passes / (time.perf_counter() - t0) / 1e9
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=262144)
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=9.0)
    args = ap.parse_args()

    import torch
    from lsbm_amd import engine, snappy
    engine.init(0)
    blocks = pool_blocks(args.pool)
    lens = np.array([len(b) for b in blocks], np.int64)
    pool = torch.from_numpy(np.frombuffer(b"".join(blocks), np.uint8).copy()).cuda()
    reps = (args.blocks + args.pool - 1) // args.pool
    n = reps * args.pool
    data = pool.repeat(reps)
    all_lens = torch.from_numpy(np.tile(lens, reps)).cuda()
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(all_lens, 0, out=offs[1:])
    raw_bytes = int(offs[-1].item())

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
        b = blocks[i % args.pool]
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
    rt_ok = bool(torch.equal(uout, data[:raw_bytes])) and int(nbad.item()) == 0
    nbad.zero_()
    t_u = timed(torch, lambda: snappy.uncompress(cdata, coffs, out=uout, out_offsets=uo, ok=ok,
                                                 n_bad=nbad), args.reps)

    cpu = cpu_baselines(blocks[:1024], args.cpu_seconds)
    alg = raw_bytes + comp_bytes
    common = {"unit": "GB/s", "higher_is_better": True, "n_gpus": 1, "dtype": "u8",
              "data": "synthetic db_bench-shaped data blocks (%d distinct, tiled), resident in HBM" % args.pool,
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
        if base in cpu:
            line["cpu_baseline"] = {"value": round(cpu[base], 3), "unit": "GB/s", "cores": 1,
                                    "kind": "libsnappy (pyarrow %s build, the library the oracle is pinned to)"
                                            % __import__("pyarrow").__version__,
                                    "sample": "1024 distinct blocks, repeated ~%.0f s" % (args.cpu_seconds / 3)}
            line["vs_cpu_core"] = round(raw_bytes / t / 1e9 / cpu[base], 1)
        if name == "snappy_compress":
            line["sample_mismatches"] = int(mism)
            line["oracle_compress_1core_GBps"] = round(cpu["oracle_compress"], 3)
        else:
            line["roundtrip_ok"] = rt_ok
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
