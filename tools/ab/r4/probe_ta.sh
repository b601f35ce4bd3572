#!/bin/bash
# Round 4: is the one-filter probe bound by its vector-memory address path?
# Lists the TA/TD/TCP counters this box has, then one PMC pass each with
# TA busy/instruction counters over the bloom probes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_probe_ta}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
echo "list rc=$?"
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/names.txt
wc -l < $OUT/names.txt
pick() { for n in "$@"; do grep -qx "$n" $OUT/names.txt && { echo -n "$n "; return; }; done; }
TA1=$(pick TA_BUSY_avr TA_TA_BUSY TA_BUSY)
TA2=$(pick TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_READ_WAVEFRONTS TA_BUFFER_READ_WAVEFRONTS_sum)
TD1=$(pick TD_BUSY_avr TD_TD_BUSY TD_BUSY)
TD2=$(pick TD_TC_STALL_sum TD_TC_STALL)
echo "counters: $TA1 $TA2 $TD1 $TD2"
[ -n "$TA1$TD1" ] || exit 0
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE $TA1 $TA2 $TD1 $TD2 \
  -d $OUT/pmc -o run -- python3 tools/bench_bloom.py build probe block --cpu-filters 0 --reps 3 > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc.log; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, collections, os, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(os.path.join(out, "pmc", "run_counter_collection.csv"))):
    if "bloom" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][-45:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(x) / len(x) for n, x in c.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 1) / 8
    print(k, " ".join("%s=%.4g" % (n, v) for n, v in sorted(m.items())), "per-XCD cycles %.0f" % cyc)
PY
