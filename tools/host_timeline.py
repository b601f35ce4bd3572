#!/usr/bin/env python3
"""Per-phase timeline of a rocprofv3 kernel + memory-copy trace of
build/bench_host_layers (tools/gpu_host_trace.sh).

Phases are told apart by the kernel they run (SSTable trailer CRCs = seal,
SSTable verify, log seal / verify); each phase is the span from its first
kernel to its last, split where kernels of one kind are more than 20 ms apart
(pageable vs page-locked runs).  For each phase: wall time, H2D bytes and
busy time (union of intervals), the longest H2D idle gaps, D2H count and busy
time, kernel busy time, and the mean per-chunk delay from an H2D's end to the
next kernel's start and from a kernel's end to its D2H's end.
"""
import csv
import glob
import os
import sys


def load(d, name):
    fs = glob.glob(os.path.join(d, "**", f"*{name}*.csv"), recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for s, e in iv:
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def kind(name):
    for tag, k in ((" 6u, 1u>", "sst_seal(trailer crcs)"), (" 3u, 1u>", "sst_verify"),
                   (" 4u, 3u>", "log_seal"), (" 5u, 3u>", "log_verify"), (" 6u, 3u>", "log_crcs")):
        if tag in name:
            return k
    return None


def main(d):
    ks = load(d, "kernel_trace")
    cs = load(d, "memory_copy_trace")
    for name, rows in (("kernel_trace", ks), ("memory_copy_trace", cs)):
        print(name, len(rows), "rows; columns:", list(rows[0].keys()) if rows else None)
    kern = []
    for r in ks:
        k = kind(r.get("Kernel_Name", ""))
        if k:
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    kern.sort()
    copies = []
    for r in cs:
        dirn = r.get("Direction", "")
        # (rocprofv3 7.2 gives no byte count: copies of >= 100 us are the bulk chunks)
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        copies.append((st, en, dirn, 1 << 30 if en - st >= 100_000 else 0))
    copies.sort()
    # phases
    phases = []
    for s, e, k in kern:
        if phases and phases[-1]["kind"] == k and s - phases[-1]["end"] < 20e6:
            p = phases[-1]
            p["end"] = max(p["end"], e)
            p["k"].append((s, e))
        else:
            phases.append({"kind": k, "start": s, "end": e, "k": [(s, e)]})
    for p in phases:
        s0, e0 = p["start"], p["end"]
        # include the H2D copies feeding the first kernel
        h2d = [c for c in copies if "HOST_TO_DEVICE" in c[2].upper() and c[1] >= s0 - 5e6 and c[0] <= e0]
        d2h = [c for c in copies if "DEVICE_TO_HOST" in c[2].upper() and c[0] >= s0 and c[0] <= e0 + 1e6]
        big = [c for c in h2d if c[3] >= (1 << 20)]
        if big:
            s0 = min(s0, big[0][0])
        wall = e0 - s0
        hb = 0
        busy = union([(c[0], c[1]) for c in h2d])
        gaps = []
        for a, b in zip(big, big[1:]):
            gaps.append(b[0] - a[1])
        gaps.sort(reverse=True)
        kb = union(p["k"])
        # per chunk: H2D (big) end -> next kernel start; kernel end -> first D2H end after it
        lag_k = []
        for c in big:
            nxt = [k for k in p["k"] if k[0] >= c[1]]
            if nxt:
                lag_k.append(nxt[0][0] - c[1])
        lag_d = []
        for k in p["k"]:
            nxt = [c for c in d2h if c[0] >= k[1]]
            if nxt:
                lag_d.append(nxt[0][1] - k[1])
        mean = lambda v: sum(v) / len(v) / 1e3 if v else 0.0
        print(f"{p['kind']:24s} kernels={len(p['k']):4d} wall={wall/1e6:8.2f} ms  "
              f"H2D busy {busy/max(wall,1)*100:5.1f}% of the wall, bulk copies={len(big)} mean {mean([c[1]-c[0] for c in big]):.0f} us, "
              f"gaps between big H2D: max {gaps[0]/1e3 if gaps else 0:.0f} us, sum {sum(gaps)/1e6:.2f} ms; "
              f"kernel busy {kb/max(wall,1)*100:4.1f}% mean {mean([k[1]-k[0] for k in p['k']]):.0f} us; "
              f"D2H n={len(d2h)} busy {union([(c[0], c[1]) for c in d2h])/1e6:.2f} ms; "
              f"H2D-end->kernel {mean(lag_k):.0f} us, kernel-end->D2H-end {mean(lag_d):.0f} us")


if __name__ == "__main__":
    main(sys.argv[1])
