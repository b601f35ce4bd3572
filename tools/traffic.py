"""Summarise a tools/gpu_profile.sh run: per-kernel average duration, HBM
traffic per launch and the derived rates; writes <out>/summary.json and the
bench's profiles/traffic.json (HBM bytes per launch of the headline kernel).

HBM bytes: MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide coalesced stream, so bytes = FETCH_SIZE * 1024 * 2;
cross-checked with TCC_EA0_RDREQ_sum * 128 B (128-B requests)."""
import collections
import csv
import json
import os
import sys

out = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEAD = "crc32c_fixed_kernel<false, 32u>"


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    p = os.path.join(d, "run_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return agg, dur


summary = {}
stats = os.path.join(out, "stats", "run_kernel_stats.csv")
for r in csv.DictReader(open(stats)):
    summary.setdefault(r["Name"], {})["avg_ns"] = float(r["AverageNs"])
    summary[r["Name"]]["calls"] = int(r["Calls"])
for i in range(1, 10):
    d = os.path.join(out, f"pmc{i}")
    if not os.path.isdir(d):
        break
    agg, dur = counters(d)
    for k, cs in agg.items():
        s = summary.setdefault(k, {})
        for c, v in cs.items():
            s[c] = sum(v) / len(v)
        if "GRBM_GUI_ACTIVE" in cs and dur[k]:
            s["clock_GHz"] = s["GRBM_GUI_ACTIVE"] / 8 / (sum(dur[k]) / len(dur[k]))
for k, s in summary.items():
    if "FETCH_SIZE" in s:
        s["hbm_read_bytes_fetch_x2"] = s["FETCH_SIZE"] * 1024 * 2
    if "TCC_EA0_RDREQ_sum" in s:
        s["hbm_read_bytes_rdreq"] = s["TCC_EA0_RDREQ_sum"] * 128
json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
head = [k for k in summary if HEAD in k]
if head:
    s = summary[head[0]]
    bytes_ = s.get("hbm_read_bytes_fetch_x2") or s.get("hbm_read_bytes_rdreq")
    t = {"workload": "1048576 x 4096 B device-resident blocks per GPU, batched crc32c::Value",
         "kernel": head[0].split("(")[0], "hbm_bytes_per_launch": bytes_,
         "hbm_bytes_rdreq_x128": s.get("hbm_read_bytes_rdreq"),
         "algorithmic_bytes_per_launch": 4294967296,
         "avg_launch_ns_rocprof": s.get("avg_ns"), "clock_GHz": s.get("clock_GHz"),
         "source": "rocprofv3 --pmc FETCH_SIZE (x1024 x2, gfx950 correction), separate pass; "
                   "tools/gpu_profile.sh"}
    json.dump(t, open(os.path.join(REPO, "profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps(t))
