#!/usr/bin/env python3
"""A whole lsbm database checked on the CPU by the reference and on the GPU
("Checking a whole database"):

    python tools/db_check_bench.py [--writes 10000000] [--runs 3]

Writes the database with the reference's own db_bench (config 1's command,
--writes), then times, on the same files (page cache warm after the first
pass of each): oracle/_ref/db_verify (the reference's ReadBlock with
verify_checksums and log::Reader, one thread: what a paranoid open /
compaction read spends on CRCs and block reads) and tools/db_check_gpu.cc
(files mapped, or read into heap buffers, every block of every table in one
VerifyTables call, logs through BatchReader; its device start-up is timed
apart).  Both must agree (no bad block, same counts).  One JSON
line per run, then a summary."""
import argparse
import json
import os
import resource
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.path.join(REPO, "oracle", "_ref")
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_ref_link import db_bench_args  # noqa: E402


def timed(cmd):
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    return r.returncode, wall, cpu, line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--writes", type=int, default=10_000_000)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    scratch = tempfile.mkdtemp(prefix="dbcheck_")
    db = os.path.join(scratch, "db")
    os.mkdir(db)
    exe = os.path.join(scratch, "db_check_gpu")
    lib = os.path.join(REPO, "lsbm_amd")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(REPO, "include"),
                    os.path.join(HERE, "db_check_gpu.cc"), "-L", lib, "-llsbm_crc32c", "-Wl,-rpath," + lib,
                    "-o", exe], check=True)
    r = subprocess.run([os.path.join(REF, "db_bench")] + db_bench_args(db, a.writes), capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = []
    for k in range(a.runs):
        rc, wall, cpu, v = timed([os.path.join(REF, "db_verify"), db])
        assert rc == 0 and not v["bad_blocks"], v
        rows.append({"run": k, "tool": "reference db_verify", "wall_ms": round(wall * 1e3, 1),
                     "cpu_ms": round(cpu * 1e3, 1), "tables": v["tables"], "blocks": v["blocks"],
                     "records": v["records"]})
        print(json.dumps(rows[-1]), flush=True)
        for mode in ("mmap", "heap"):
            rc, wall, cpu, g = timed([exe, db, "0"] + (["--read=heap"] if mode == "heap" else []))
            assert rc == 0 and not g["bad_blocks"] and g["blocks"] == v["blocks"] and g["records"] == v["records"], g
            rows.append({"run": k, "tool": "db_check_gpu", "read": mode, "wall_ms": round(wall * 1e3, 1),
                         "cpu_ms": round(cpu * 1e3, 1), "device_init_ms": g["device_init_ms"],
                         "tables": g["tables"], "blocks": g["blocks"], "table_bytes": g["table_bytes"],
                         "records": g["records"], "log_bytes": g["log_bytes"], "read_parse_ms": g["read_parse_ms"],
                         "verify_tables_ms": g["verify_tables_ms"],
                         "verify_tables_again_ms": g["verify_tables_again_ms"], "logs_ms": g["logs_ms"],
                         "check_ms": g["total_ms"], "check_cpu_ms": g["host_cpu_ms"],
                         "verify_tables_again_GBps": round(g["table_bytes"] / (g["verify_tables_again_ms"] * 1e-3) / 1e9,
                                                           1)})
            print(json.dumps(rows[-1]), flush=True)
    # and once with every table's filter block rebuilt: by the reference's own
    # FilterBlockBuilder on one core, and on the GPU (then every key probed)
    rc, wall, cpu, v = timed([os.path.join(REF, "db_verify"), db, "--filters"])
    assert rc == 0 and v["filters_identical"] == v["filters_rebuilt"], v
    rows.append({"tool": "reference db_verify --filters", "filters_rebuilt": v["filters_rebuilt"],
                 "filters_identical": v["filters_identical"], "filters_ms": v["filters_ms"]})
    print(json.dumps(rows[-1]), flush=True)
    rc, wall, cpu, g = timed([exe, db, "0", "--filters"])
    assert rc == 0 and g["filters_identical"] == g["filters_rebuilt"] == g["tables"] and g["false_negatives"] == 0, g
    rows.append({"tool": "db_check_gpu --filters", "filters_rebuilt": g["filters_rebuilt"],
                 "filters_identical": g["filters_identical"], "keys_probed": g["keys_probed"],
                 "false_negatives": g["false_negatives"], "filters_build_ms": g["filters_build_ms"],
                 "filters_feed_ms": g["filters_feed_ms"], "filters_finish_ms": g["filters_finish_ms"],
                 "filters_probe_ms": g["filters_probe_ms"]})
    print(json.dumps(rows[-1]), flush=True)
    ref = [r for r in rows if r["tool"] == "reference db_verify"]
    summary = {"writes": a.writes, "reference_wall_ms_best": min(r["wall_ms"] for r in ref)}
    for mode in ("mmap", "heap"):
        g = [r for r in rows if r.get("read") == mode]
        summary[mode] = {"check_ms_best": min(r["check_ms"] for r in g),
                         "verify_tables_ms_best": min(r["verify_tables_ms"] for r in g),
                         "verify_tables_again_ms_best": min(r["verify_tables_again_ms"] for r in g),
                         "device_init_ms_best": min(r["device_init_ms"] for r in g),
                         "wall_ms_best": min(r["wall_ms"] for r in g)}
    print(json.dumps({"summary": summary}), flush=True)
    shutil.rmtree(scratch, ignore_errors=True)


if __name__ == "__main__":
    main()
