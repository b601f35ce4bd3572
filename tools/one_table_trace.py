#!/usr/bin/env python3
"""Summary of a rocprofv3 kernel + memory-copy + HIP-runtime trace of
build/bench_one_table (tools/r4/one_table.sh): the longest HIP API calls (with
their time after the process's first kernel launch), and the timeline of one
call of each kind -- API calls, copies and kernels relative to the call's first
API call -- so the per-call costs (enqueue, DMA, kernel, syncs, host gaps) can
be read off.

    python3 tools/one_table_trace.py <trace dir> [call index]
"""
import csv
import glob
import os
import sys


def load(d, name):
    rows = []
    for f in glob.glob(os.path.join(d, "**", f"*{name}*.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(d, pick=100):
    api = load(d, "hip_api_trace")
    cps = load(d, "memory_copy_trace")
    ks = load(d, "kernel_trace")
    if not api:
        print("no hip_api_trace under", d)
        return 1
    t_launch = min(int(r["Start_Timestamp"]) for r in api if r["Function"] == "hipLaunchKernel")
    dur = sorted(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r) for r in api), key=lambda x: -x[0])
    print("longest HIP API calls (ms; start ms after the first kernel launch):")
    for dt, r in dur[:15]:
        print(f"  {dt / 1e6:9.3f}  {r['Function']:<26} corr {r['Correlation_Id']:>6}  at "
              f"{(int(r['Start_Timestamp']) - t_launch) / 1e6:9.3f}")
    # one call: the pick-th hipPointerGetAttributes (each layer call starts with
    # host_pinned's attribute queries) to the next one
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", r["Function"], r["Correlation_Id"]) for r in api]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "CPY",
            r["Direction"].replace("MEMORY_COPY_", "") + " s" + r["Stream_Id"], r["Correlation_Id"]) for r in cps]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "KER",
            r["Kernel_Name"].split("(")[0][-40:] + " s" + r["Stream_Id"], r["Correlation_Id"]) for r in ks]
    ev.sort()
    # a call starts with host_pinned's attribute queries (one for a pageable
    # image, two or three for a page-locked one): the first of a run of them
    apis = [e for e in ev if e[2] == "API"]
    starts = [e[0] for i, e in enumerate(apis)
              if e[3] == "hipPointerGetAttributes" and (i == 0 or apis[i - 1][3] != "hipPointerGetAttributes")]
    if len(starts) > pick + 1:
        t0, t1 = starts[pick], starts[pick + 1]
        print(f"\ntimeline of call {pick} ({(t1 - t0) / 1e3:.1f} us to the next call), us from its start:")
        for e in ev:
            if t0 <= e[0] < t1:
                print(f"  {(e[0] - t0) / 1e3:8.1f} {(e[1] - e[0]) / 1e3:8.1f}  {e[2]} {e[3]} {e[4]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100))
