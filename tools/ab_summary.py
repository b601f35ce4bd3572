#!/usr/bin/env python3
"""One line per (log, workload) of tools/bench_configs.py output: % of HBM peak."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        c = d["config"]
        if c == "wal":
            r = {k: d[k]["pct_hbm_peak"] for k in ("log_seal", "log_seal_no_out", "log_crcs", "log_verify") if k in d}
        elif c == "sst4118":
            r = {"ext": d["pct_hbm_peak"], "seal": d["sst_seal"]["pct_hbm_peak"],
                 "tcrc": d["sst_trailer_crcs"]["pct_hbm_peak"], "verify": d["sst_verify"]["pct_hbm_peak"]}
        else:
            r = {"pct": d.get("pct_hbm_peak")}
        bad = d.get("sample_mismatches", 0)
        print(f"{f.split('/')[-1]:22s} {c:9s} " + " ".join(f"{k}={v}" for k, v in r.items()) + (f" MISMATCH={bad}" if bad else ""))
