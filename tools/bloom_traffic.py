#!/usr/bin/env python3
"""HBM bytes per launch of the bloom kernels from tools/gpu_bloom_traffic.sh's
PMC passes -> profiles/bloom_traffic.json (read by tools/bench_bloom.py).

Reads: FETCH_SIZE (KiB) x 1024 x 2, the gfx950 correction of
MI355X_MICROARCH.md "HBM" (FETCH_SIZE reports half the bytes of a wide
coalesced stream).  Round 4 calibrated the probes' scattered 1-4 B reads on a
known line count (tools/fetch_calib.hip, profiles/r04/fetch_calib/): every
width goes to memory as one request per 128-B line, tallied at 64 B, so the
same x2 gives their fetched line bytes; the raw x1 figure is kept beside it.
Writes: WRITE_SIZE (KiB) x 1024, exact for streaming stores."""
import collections
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def name_of(k):
    if "bloom_build_kernel" in k:
        return "bloom_build"
    if "bloom_probe_kernel" in k:
        # one instantiation per mode (bloom_types.h: 0 one filter, 1 filter block)
        return "bloom_block" if k.split("bloom_probe_kernel")[1].startswith("<1") else "bloom_probe"
    return None


res = collections.defaultdict(dict)
names = set()
for d in sorted(glob.glob(os.path.join(out, "p*"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            names.add(r["Kernel_Name"])
            k = name_of(r["Kernel_Name"])
            if k:
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in agg.items():
            res[k][c] = sum(v) / len(v)
summary = {}
for k, s in res.items():
    e = {}
    if "FETCH_SIZE" in s:
        e["read_bytes_fetch_x2"] = s["FETCH_SIZE"] * 1024 * 2
        e["read_bytes_fetch_x1"] = s["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in s:
        e["write_bytes"] = s["WRITE_SIZE"] * 1024
    if "read_bytes_fetch_x2" in e:
        e["traffic"] = e["read_bytes_fetch_x2"] + e.get("write_bytes", 0.0)
    summary[k] = e
summary["_kernels_seen"] = sorted(n.split("(")[0] for n in names)
summary["_note"] = ("per launch; reads FETCH_SIZE x 2 (gfx950 stream correction), writes WRITE_SIZE; "
                    "tools/gpu_bloom_traffic.sh")
json.dump(summary, open(os.path.join(REPO, "profiles", "bloom_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
