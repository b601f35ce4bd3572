#!/usr/bin/env python3
"""Config 1 measured with lsbm's own db_bench, three builds interleaved
(oracle/Makefile dbbench_gpu; DESIGN.md section 5, "db_bench end to end"):

    python tools/db_bench_ab.py [--passes 5] [--writes 1000000] [--scratch DIR]

  ref   oracle/_ref/db_bench      the reference as shipped (slice-by-4 CRC on the CPU)
  l1    oracle/_ref/db_bench_l1   Level 1: Extend / Hash from liblsbm_crc32c.so
  gpu   oracle/_ref/db_bench_gpu  Level 2: also every table sealed on the GPU
                                  (integration/table_builder_gpu.cc)
  gpu_unlocked                    the same with the pooled images not kept
                                  page-locked (LSBM_TABLE_REGISTER=0)

Per run: db_bench's own report (micros/op of the writer thread over the 1M
writes), the process's wall time and CPU time (user + sys of all its
threads: the reaped child's rusage), and for the GPU build the tables it sealed.
Every database is checked afterwards by oracle/_ref/db_verify (reference code
only: every block and log record verified).  One JSON line per run, then a
summary line with the medians.
"""
import argparse
import json
import os
import resource
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.path.join(REPO, "oracle", "_ref")
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_ref_link import db_bench_args  # noqa: E402

BUILDS = {"ref": ("db_bench", {}), "l1": ("db_bench_l1", {}), "gpu": ("db_bench_gpu", {}),
          "gpu_unlocked": ("db_bench_gpu", {"LSBM_TABLE_REGISTER": "0"})}


def run(build, writes, scratch):
    db = tempfile.mkdtemp(prefix=f"dbab_{build}_", dir=scratch)
    exe, extra = BUILDS[build]
    env = dict(os.environ, LSBM_TABLE_STATS="1", **extra)
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    p = subprocess.Popen([os.path.join(REF, exe)] + db_bench_args(db, writes),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    out, err = p.communicate(timeout=600)  # (reaped: its rusage is in RUSAGE_CHILDREN now)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    rc = p.returncode
    line = [ln for ln in out.splitlines() if ln.startswith("separate")]
    us = float(line[0].split(":")[1].split("micros/op")[0]) if line else None
    stats = [ln for ln in err.splitlines() if ln.startswith("lsbm_table_stats")]
    v = subprocess.run([os.path.join(REF, "db_verify"), db], capture_output=True, text=True, timeout=600)
    vj = json.loads([ln for ln in v.stdout.splitlines() if ln.startswith("{")][-1])
    shutil.rmtree(db, ignore_errors=True)
    return {"build": build, "rc": rc, "micros_per_op": us, "wall_s": round(wall, 3), "cpu_s": round(cpu, 3),
            "stats": stats,
            "verify_rc": v.returncode, "tables": vj["tables"], "table_errors": vj["table_errors"],
            "log_errors": vj["log_errors"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--writes", type=int, default=1_000_000)
    ap.add_argument("--scratch", default=tempfile.gettempdir())
    a = ap.parse_args()
    rows = []
    for p in range(a.passes):
        for b in BUILDS:
            row = run(b, a.writes, a.scratch)
            row["pass"] = p
            rows.append(row)
            print(json.dumps(row), flush=True)
            if row["rc"] != 0 or row["verify_rc"] != 0:
                sys.exit(1)
    summary = {}
    for b in BUILDS:
        rs = [r for r in rows if r["build"] == b]
        summary[b] = {"micros_per_op_median": statistics.median(r["micros_per_op"] for r in rs),
                      "micros_per_op_min": min(r["micros_per_op"] for r in rs),
                      "wall_s_median": statistics.median(r["wall_s"] for r in rs),
                      "cpu_s_median": statistics.median(r["cpu_s"] for r in rs)}
    print(json.dumps({"summary": summary, "writes": a.writes, "passes": a.passes}), flush=True)


if __name__ == "__main__":
    main()
