#!/bin/bash
# Round 4: bloom build, in-tree (carried key extents, single-compare masks,
# scalar span tests, the hash tail's bytes in one step) against two register
# sets alternating between rounds (build/abl/pp, without the tail change) and
# the kernels before (build/abl/r4base); then one PMC pass per variant for
# VALU instructions per round.  Bloom tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check27}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom.log 2>&1
rc=$?; echo "bloom tests rc=$rc"; tail -1 $OUT/pytest_bloom.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default pp r4base; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py build probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
for v in default r4base; do
  if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
  LSBM_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    -d $OUT/pmc_$v -o run -- python3 tools/bench_bloom.py build --cpu-filters 0 --reps 3 > $OUT/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, collections, os, sys
out = sys.argv[1]
for v in ("default", "r4base"):
    c = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(out, "pmc_" + v, "run_counter_collection.csv"))):
        if "bloom_build" in r["Kernel_Name"]:
            c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {n: sum(x) / len(x) for n, x in c.items()}
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    print(v, "VALU/round %.1f SALU/round %.1f LDS/round %.1f VALU issue/SIMD-cycle %.3f wait %.2f" % (
        m["SQ_INSTS_VALU"] / 524288, m["SQ_INSTS_SALU"] / 524288, m["SQ_INSTS_LDS"] / 524288,
        m["SQ_INSTS_VALU"] / (1024 * cyc), m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]))
PY
