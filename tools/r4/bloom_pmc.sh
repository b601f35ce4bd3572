#!/bin/bash
# Round 4: PMC passes over the bloom kernels as they stand (build, probe,
# filter-block probe): issue (VALU / SALU / LDS / VMEM counts), waits, LDS
# bank conflicts.  One rocprofv3 run per counter group.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_bloom_pmc}
mkdir -p $OUT
CMD="python3 tools/bench_bloom.py build probe block --cpu-filters 0 --reps 3"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, collections, json, sys, os
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(os.listdir(out)):
    p = os.path.join(out, d, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "bloom" not in k:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, c in agg.items():
    res[k] = {n: sum(v) / len(v) for n, v in c.items()}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k, c in res.items():
    print(k[:80])
    print("  " + ", ".join("%s=%.4g" % (n, v) for n, v in sorted(c.items())))
PY
