#!/bin/bash
# Round 4: PMC of the probe kernels, in-tree against the 32-bit fast lookup
# (build/abl/fast, commit 826b9b9's kernels): does ~80 fewer VALU per round
# change the issue picture?
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_bloom_pmc_ab}
mkdir -p $OUT
for v in default fast; do
  if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    LSBM_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $OUT/${v}_p$i -o run -- python3 tools/bench_bloom.py probe block --cpu-filters 0 --reps 3 > $OUT/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 - "$OUT" <<'PY'
import csv, collections, os, sys
out = sys.argv[1]
for v in ("default", "fast"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for i in (1, 2):
        p = os.path.join(out, "%s_p%d" % (v, i), "run_counter_collection.csv")
        for r in csv.DictReader(open(p)):
            if "bloom_probe" in r["Kernel_Name"]:
                agg[r["Kernel_Name"][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        m = {n: sum(x) / len(x) for n, x in c.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 1) / 8
        print(v, k, "VALU/round %.0f SALU/round %.0f VALU busy %.2f wait %.2f cycles/XCD %.0f" % (
            m["SQ_INSTS_VALU"] / 524288, m["SQ_INSTS_SALU"] / 524288, m["SQ_INSTS_VALU"] / (256 * cyc),
            m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], cyc))
PY
