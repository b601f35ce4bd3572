#!/usr/bin/env python3
"""Join tools/roofline.sh's passes per entry (tools/roofline_all.py):
rocprof's average duration of the entry's kernel(s) (kernel-trace stats),
its HBM read bytes per dispatch (FETCH_SIZE x 1024 x 2, the gfx950
correction of MI355X_MICROARCH.md) and the entry's algorithmic bytes.

  roofline_summary.py OUT ENTRY   -> OUT/ENTRY/summary.json (and compacts the PMC CSV)
  roofline_summary.py OUT         -> OUT/summary.json + OUT/table.md over every entry
"""
import collections
import csv
import json
import os
import re
import sys

PEAK = 8000.0  # GB/s


def one(out, e):
    d = os.path.join(out, e)
    meta = [json.loads(l) for l in open(os.path.join(d, "stats.log")) if l.startswith('{"entry"')][0]
    rx = re.compile(meta["kernel_regex"])
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "stats", "run_kernel_stats.csv"))):
        if rx.search(r["Name"]):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                "total_ns": float(r["TotalDurationNs"])}
    fetch = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    p = os.path.join(d, "pmc", "run_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            if rx.search(r["Kernel_Name"]) and r["Counter_Name"] == "FETCH_SIZE":
                fetch[r["Kernel_Name"]] += float(r["Counter_Value"])
                disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
        for k in fetch:
            stats.setdefault(k, {})["hbm_read_bytes"] = fetch[k] / len(disp[k]) * 1024 * 2
    elif os.path.exists(os.path.join(d, "summary.json")):
        return json.load(open(os.path.join(d, "summary.json")))
    # the entry's device time per call: every matching kernel's total over the
    # calls of the one with the most time (the main kernel; a pre-pass adds its share)
    main = max(stats, key=lambda k: stats[k].get("total_ns", 0))
    calls = stats[main]["calls"]
    ns = sum(s.get("total_ns", 0) for s in stats.values()) / calls
    read = sum(s.get("hbm_read_bytes", 0) for s in stats.values())
    alg = meta["algorithmic_bytes"]
    res = {"entry": e, "kernel": main, "kernels": stats, "calls": calls, "avg_ms_rocprof": round(ns / 1e6, 4),
           "algorithmic_bytes": alg, "achieved_GBps": round(alg / ns, 1), "frac_of_8TBps": round(alg / ns / PEAK, 4),
           "hbm_read_over_algorithmic": round(read / alg, 4) if read else None,
           "events_ms": meta["events_ms"], "sample_mismatches": meta["sample_mismatches"]}
    json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(f"{e}: {res['avg_ms_rocprof']} ms, {res['achieved_GBps']} GB/s = {100 * res['frac_of_8TBps']:.1f}%, "
          f"HBM reads {res['hbm_read_over_algorithmic']}x algorithmic")
    return res


def main():
    out = sys.argv[1]
    if len(sys.argv) > 2:
        one(out, sys.argv[2])
        return
    rows = []
    for e in sorted(os.listdir(out)):
        if os.path.exists(os.path.join(out, e, "summary.json")):
            rows.append(json.load(open(os.path.join(out, e, "summary.json"))))
    json.dump(rows, open(os.path.join(out, "summary.json"), "w"), indent=1)
    with open(os.path.join(out, "table.md"), "w") as f:
        f.write("| entry | kernel | rocprof avg ms | algorithmic GB | GB/s | % of 8 TB/s | HBM reads / algorithmic |\n")
        f.write("|---|---|---|---|---|---|---|\n")
        for r in rows:
            k = re.sub(r"^void lsbm::|\(.*$", "", r["kernel"])
            f.write(f"| {r['entry']} | `{k}` | {r['avg_ms_rocprof']} | {r['algorithmic_bytes'] / 1e9:.3f} | "
                    f"{r['achieved_GBps']} | {100 * r['frac_of_8TBps']:.1f} | {r['hbm_read_over_algorithmic']} |\n")
    print(open(os.path.join(out, "table.md")).read())


if __name__ == "__main__":
    main()
