#!/usr/bin/env python3
"""Bloom-filter rates on one GPU, db_bench shaped:
internal keys "user%019d" + 8-byte sequence/type (31 B, lsbm/db_bench.cc:1415),
33 keys per filter (one ~4 KiB data block per 2 KiB filter slot,
table/filter_block.cc:14-16), BloomFilterPolicy(20) under InternalFilterPolicy
(strip 8), config::bloom_bits_use = 15.  Keys are generated on the device and
resident in HBM before timing.  One JSON line per measurement:

  bloom_build   lsbm_bloom_build_dev over every filter of the batch
  bloom_probe   lsbm_bloom_may_match_dev, every key against its own filter
  bloom_block   lsbm_filter_block_may_match_dev, through FilterBlockReader's
                offset array (one filter block per 1,024 filters)

Algorithmic bytes are stated per line.  The build's roofline fraction uses
them (its counter bytes are >= them); the probes are reported as queries per
second and 128-B HBM lines fetched per query (calibrated PMC counters,
profiles/bloom_traffic.json), with no % of HBM: their queries share filter
lines, so counter bytes fall below the byte model, and they are bound by
dependent-load latency, not bandwidth.
cpu_baseline: the reference's own CreateFilter / KeyMayMatch
(oracle/_ref/libref_bloom.so, built from /root/reference) on every usable
host core and on one, on a bounded sample, else the oracle's C restatement.
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
sys.path.insert(0, os.path.join(REPO, "tests"))

HBM = 8000.0  # GB/s, MI355X spec
KLEN, PER, BPK = 31, 33, int(os.environ.get("LSBM_BENCH_BPK", "20"))  # (env: diagnostic k sweeps)


def dbbench_keys_dev(torch, n, first=0, seq0=1):
    nums = torch.arange(first, first + n, dtype=torch.int64, device="cuda")
    out = torch.empty((n, KLEN), dtype=torch.uint8, device="cuda")
    out[:, :4] = torch.tensor(list(b"user"), dtype=torch.uint8, device="cuda")
    for p in range(19):
        out[:, 4 + p] = (torch.div(nums, 10 ** (18 - p), rounding_mode="floor") % 10 + 48).to(torch.uint8)
    tag = (torch.arange(seq0, seq0 + n, dtype=torch.int64, device="cuda") << 8) | 1
    for b in range(8):
        out[:, 23 + b] = ((tag >> (8 * b)) & 0xFF).to(torch.uint8)
    return out.reshape(-1)


def timed(torch, fn, reps, warm=2, spin_s=None):
    """Seconds per call, after spin_s seconds of untimed calls: after a host
    pause the GPU clock has dropped.  LSBM_SPIN_S=0
    under rocprofv3 --pmc."""
    if spin_s is None:
        spin_s = float(os.environ.get("LSBM_SPIN_S", "0.3"))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < spin_s:
        for _ in range(10):
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


def cpu_baseline(sample_filters, seconds=4.0):
    """The reference's own CreateFilter / KeyMayMatch loops (C) on a bounded
    db_bench-shaped sample, repeated for about `seconds`, on every usable host
    core (one thread each: ctypes releases the GIL, every thread has its own
    output), plus the one-core rate; the oracle's C restatement on one core
    when the reference build is absent."""
    import threading
    from golden.bloomkeys import dbbench_keys
    sys.path.insert(0, REPO)
    from bench import usable_cores
    n = sample_filters * PER
    first = np.minimum(np.arange(sample_filters + 1, dtype=np.uint64) * PER, n).astype(np.uint64)
    fidx = (np.arange(n) // PER).astype(np.uint64)
    fo = np.zeros(sample_filters + 1, dtype=np.uint64)
    out = np.zeros(sample_filters * 100, dtype=np.uint8)
    vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    ref = os.path.join(REPO, "oracle", "_ref", "libref_bloom.so")
    threads = 1
    if os.path.exists(ref):
        lib, kind = ctypes.CDLL(ref), "reference"
        lib.ref_create_filters.restype = sz
        lib.ref_create_filters.argtypes = [i32, vp, vp, vp, sz, vp, vp]
        lib.ref_may_match_batch.restype = sz
        lib.ref_may_match_batch.argtypes = [i32, vp, vp, sz, vp, vp, vp]
        # InternalFilterPolicy hands the bloom policy user keys: 23 B
        keys, offs = dbbench_keys(0, n, internal=False)
        threads = usable_cores()[0]
        outs = [np.zeros_like(out) for _ in range(threads)]
        fos = [np.zeros_like(fo) for _ in range(threads)]

        def build(t=0):
            lib.ref_create_filters(BPK, keys.ctypes.data, offs.ctypes.data, first.ctypes.data,
                                   sample_filters, outs[t].ctypes.data, fos[t].ctypes.data)

        def probe(t=0):
            return lib.ref_may_match_batch(BPK, keys.ctypes.data, offs.ctypes.data, n,
                                           outs[0].ctypes.data, fos[0].ctypes.data, fidx.ctypes.data)
    else:
        from conftest import BloomOracle
        o = BloomOracle(os.path.join(REPO, "oracle", "liboracle_bloom.so"))
        kind = "port"
        keys, offs = dbbench_keys(0, n)
        fsize = o.filter_bytes(PER, BPK)
        fo[:] = np.arange(sample_filters + 1, dtype=np.uint64) * fsize

        def build(t=0):
            for f in range(sample_filters):
                o.lib.bo_create_filter(keys.ctypes.data, offs[f * PER:].ctypes.data, PER, 8, BPK,
                                       out.ctypes.data + f * fsize)

        def probe(t=0):
            return sum(o.lib.bo_key_may_match(keys.ctypes.data + int(offs[i]), KLEN, 8,
                                              out.ctypes.data + int(fidx[i]) * fsize, fsize, BPK, 15)
                       for i in range(n))

    def rate(fn, nt):
        """keys per second over nt threads, each repeating fn for ~seconds / 4"""
        reps = [0] * nt
        res = [None] * nt
        go = threading.Barrier(nt + 1)

        def worker(t):
            go.wait()
            t0 = time.perf_counter()
            while True:
                res[t] = fn(t)
                reps[t] += 1
                if time.perf_counter() - t0 >= seconds / 4:
                    return
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(nt)]
        for th in ths:
            th.start()
        go.wait()
        t0 = time.perf_counter()
        for th in ths:
            th.join()
        return sum(reps) * n / (time.perf_counter() - t0), res[0]
    build(0)  # the filters probe() reads
    build_1, _ = rate(build, 1)
    probe_1, hits = rate(probe, 1)
    build_all, _ = rate(build, threads) if threads > 1 else (build_1, None)
    probe_all, _ = rate(probe, threads) if threads > 1 else (probe_1, None)
    cpu = ""
    try:
        cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except (OSError, IndexError):
        pass
    return {"kind": kind, "cores": threads, "build_keys_per_s": round(build_all, 1),
            "probe_keys_per_s": round(probe_all, 1), "build_keys_per_s_1core": round(build_1, 1),
            "probe_keys_per_s_1core": round(probe_1, 1), "members_found": int(hits) == n,
            "sample": f"{sample_filters} filters x {PER} db_bench keys, CreateFilter and "
                      f"KeyMayMatch loops in C, {threads} thread(s) (every usable core) and 1, "
                      f"~{seconds:.0f} s; {cpu}"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", nargs="*", default=["build", "probe", "block"])
    p.add_argument("--keys", type=int, default=1 << 25)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--cpu-filters", type=int, default=20000)
    args = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from conftest import BloomOracle
    from golden.bloomkeys import dbbench_keys, take
    from lsbm_amd import bloom, engine
    engine.init(0)
    o = BloomOracle(os.path.join(REPO, "oracle", "liboracle_bloom.so"))
    n = args.keys
    nf = (n + PER - 1) // PER
    keys = dbbench_keys_dev(torch, n)
    koffs = torch.arange(0, (n + 1) * KLEN, KLEN, dtype=torch.int64, device="cuda")
    first = torch.clamp(torch.arange(0, nf + 1, dtype=torch.int64, device="cuda") * PER, max=n)
    counts = (first[1:] - first[:-1]).cpu().numpy()
    fbytes = np.array([bloom.filter_bytes(c, BPK) for c in np.unique(counts)])
    size_of = dict(zip(np.unique(counts).tolist(), fbytes.tolist()))
    sizes = np.array([size_of[c] for c in counts.tolist()], dtype=np.int64)
    outo_h = np.zeros(nf, dtype=np.int64)
    outo_h[1:] = np.cumsum(sizes)[:-1]
    outo = torch.from_numpy(outo_h).to("cuda")
    total_out = int(sizes.sum())
    out = torch.empty(total_out, dtype=torch.uint8, device="cuda")
    lines = []

    def build():
        bloom.build_filters(keys, koffs, first, outo, out, BPK, strip=8)

    t = timed(torch, build, args.reps)
    host_out = out.cpu().numpy()
    rng = np.random.default_rng(9)
    bad = 0
    hk = None
    for f in rng.choice(nf, 32, replace=False):
        k0, k1 = int(f) * PER, min(n, int(f) * PER + PER)
        want = o.create_filter(dbbench_keys(k0, k1 - k0, seq0=1 + k0), BPK, 8)
        bad += int(host_out[outo_h[f]:outo_h[f] + sizes[f]].tobytes() != want)
    alg = n * KLEN + (n + 1) * 8 + nf * 16 + total_out
    gbps = alg / t / 1e9
    lines.append({"bench": "bloom_build", "keys": n, "filters": nf, "keys_per_filter": PER,
                  "bits_per_key": BPK, "ms": round(t * 1e3, 3), "Gkeys_per_s": round(n / t / 1e9, 2),
                  "algorithmic_bytes": alg, "GBps": round(gbps, 1),
                  "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM,
                               "unit": "GB/s", "frac": round(gbps / HBM, 4)},
                  "bytes_note": "31 B key + 8 B key offset per key, 16 B per filter, filter bytes written",
                  "sample_mismatches": bad})
    fidx = torch.div(torch.arange(n, device="cuda"), PER, rounding_mode="floor")
    sizes_d = torch.from_numpy(sizes).to("cuda")
    handles = torch.stack([outo[fidx], sizes_d[fidx]], 1).reshape(-1).contiguous()
    if "probe" in args.which:
        may = torch.empty(n, dtype=torch.uint8, device="cuda")
        n_may = torch.zeros(1, dtype=torch.int32, device="cuda")

        def probe():
            bloom.may_match(out, handles, keys, koffs, BPK, 15, strip=8, may=may, n_may=n_may)

        t = timed(torch, probe, args.reps)
        n_may.zero_()
        probe()
        found = int(n_may.item())
        alg = n * (KLEN + 8 + 16 + 1 + bloom.k_probe(BPK, 15))
        gbps = alg / t / 1e9
        lines.append({"bench": "bloom_probe", "queries": n, "ms": round(t * 1e3, 3),
                      "Gqueries_per_s": round(n / t / 1e9, 2), "algorithmic_bytes": alg,
                      "GBps": round(gbps, 1),
                      "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM,
                                   "unit": "GB/s", "frac": round(gbps / HBM, 4)},
                      "bytes_note": "31 B key + 8 B offset + 16 B handle + 1 B result + k_use probe bytes",
                      "members_found": found, "no_false_negatives": found == n})
    if "block" in args.which:
        # filter blocks of 1,024 filters each: data blocks at 4,096-B strides
        per_blk = 1024
        nb = (nf + per_blk - 1) // per_blk
        blocks, bh = [], []
        pos = 0
        for b in range(nb):
            f0, f1 = b * per_blk, min(nf, b * per_blk + per_blk)
            data = host_out[outo_h[f0]:outo_h[f1 - 1] + sizes[f1 - 1]]
            offsets = (outo_h[f0:f1] - outo_h[f0]).astype("<u4")
            # one 4 KiB data block per filter: filter index = 2 per data block
            arr = np.zeros(2 * (f1 - f0), dtype="<u4")
            arr[0::2] = offsets
            arr[1::2] = np.append(offsets[1:], data.size).astype("<u4")  # odd slots: empty filters
            tail = np.frombuffer(np.uint32(data.size).tobytes() + bytes([11]), np.uint8)
            blk = np.concatenate([data, arr.view(np.uint8), tail])
            blocks.append(blk)
            bh.append((pos, blk.size))
            pos += blk.size
        blob = torch.from_numpy(np.concatenate(blocks)).to("cuda")
        qb = (fidx // per_blk).cpu().numpy()
        bhn = np.array(bh, dtype=np.int64)
        bhandles = torch.from_numpy(bhn[qb].reshape(-1).copy()).to("cuda")
        doffs = ((fidx % per_blk) * 4096).to(torch.int64)
        may = torch.empty(n, dtype=torch.uint8, device="cuda")
        n_may = torch.zeros(1, dtype=torch.int32, device="cuda")

        def block():
            bloom.filter_block_may_match(blob, bhandles, doffs, keys, koffs, BPK, 15, strip=8,
                                         may=may, n_may=n_may)

        t = timed(torch, block, args.reps)
        n_may.zero_()
        block()
        found = int(n_may.item())
        alg = n * (KLEN + 8 + 16 + 8 + 1 + 8 + 1 + bloom.k_probe(BPK, 15))
        gbps = alg / t / 1e9
        lines.append({"bench": "bloom_block", "queries": n, "filter_blocks": nb,
                      "ms": round(t * 1e3, 3), "Gqueries_per_s": round(n / t / 1e9, 2),
                      "algorithmic_bytes": alg, "GBps": round(gbps, 1),
                      "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM,
                                   "unit": "GB/s", "frac": round(gbps / HBM, 4)},
                      "bytes_note": "key + offset + block handle + data offset + trailer byte "
                                    "+ 2 offset words + k byte + k_use probe bytes",
                      "members_found": found, "no_false_negatives": found == n})
    cpu = cpu_baseline(args.cpu_filters) if args.cpu_filters else None
    # HBM bytes per launch from the PMC passes of tools/gpu_bloom_traffic.sh (same workload)
    tp = os.path.join(REPO, "profiles", "bloom_traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    for ln in lines:
        t = traffic.get(ln["bench"], {}).get("traffic")
        ln["roofline"]["traffic"] = int(t) if t else None
        if t:
            ln["roofline"]["traffic_over_algorithmic"] = round(t / ln["algorithmic_bytes"], 3)
            # FETCH_SIZE x 2 is the fetched line bytes for every access width on
            # gfx950, these scattered reads included (tools/fetch_calib.hip:
            # one memory request per 128-B line, profiles/r04/fetch_calib/)
            ln["roofline"]["traffic_calibration"] = "profiles/r04/fetch_calib/summary.json"
        q = ln.get("queries")
        if t and q:
            # Probes: queries per second and the 128-B lines each one fetches
            # from HBM (calibrated counters).  Queries share filter lines, so
            # the counters see fewer bytes than the byte model counts: a % of
            # HBM from algorithmic bytes would overstate these kernels, which
            # PMC shows bound by dependent-load latency.
            # A % of HBM is reported only where counter bytes >= algorithmic.
            secs = ln["ms"] / 1e3
            ln["lines_128B_per_query"] = round(t / 128 / q, 3)
            ln["hbm_GBps_by_counters"] = round(t / secs / 1e9, 1)
            if t < ln["algorithmic_bytes"]:
                ln["roofline"] = {"bound": "latency (dependent loads: key -> hash -> filter line)",
                                  "frac": None, "hbm_frac_by_counters": round(t / secs / 1e9 / HBM, 4),
                                  "traffic": int(t), "traffic_over_algorithmic": round(t / ln["algorithmic_bytes"], 3),
                                  "algorithmic_GBps_not_a_roofline": ln["GBps"],
                                  "traffic_calibration": "profiles/r04/fetch_calib/summary.json"}
        if cpu:
            ln["cpu_baseline"] = cpu
        print(json.dumps(ln), flush=True)


if __name__ == "__main__":
    main()
