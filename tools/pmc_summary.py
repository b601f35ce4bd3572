"""Summarise tools/gpu_units_pmc.sh output: per kernel, the rocprof average
duration (kernel-trace stats) and the PMC counters averaged per dispatch,
plus HBM bytes (MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half of a
wide coalesced read, so read bytes = FETCH_SIZE x 1024 x 2; cross-checked with
TCC_EA0_RDREQ x 128 B) and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / t).
Writes <dir>/summary.json and prints one line per kernel."""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
summary = collections.OrderedDict()
for r in csv.DictReader(open(os.path.join(d, "stats", "run_kernel_stats.csv"))):
    summary[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
for i in range(1, 10):
    p = os.path.join(d, f"pmc{i}", "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, cs in vals.items():
        s = summary.setdefault(k, {})
        for c, v in cs.items():
            s[c] = v / len(disp[k])
for k, s in summary.items():
    if "FETCH_SIZE" in s:
        s["hbm_read_bytes"] = s["FETCH_SIZE"] * 1024 * 2
    if "TCC_EA0_RDREQ_sum" in s:
        s["hbm_read_bytes_rdreq"] = s["TCC_EA0_RDREQ_sum"] * 128
    if "WRITE_SIZE" in s:
        s["hbm_write_bytes"] = s["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in s and s.get("avg_ns"):
        s["clock_GHz"] = s["GRBM_GUI_ACTIVE"] / 8 / s["avg_ns"]
json.dump(summary, open(os.path.join(d, "summary.json"), "w"), indent=1)
for k, s in summary.items():
    short = k.split("(")[0][-70:]
    keys = ["calls", "avg_ns", "hbm_read_bytes", "hbm_write_bytes", "clock_GHz", "SQ_INSTS_VALU",
            "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES"]
    print(short, {x: (round(s[x], 3) if isinstance(s[x], float) else s[x]) for x in keys if x in s})
