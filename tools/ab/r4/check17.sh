#!/bin/bash
# Round 4: what page-locking an image per call costs (THP-backed and 4 KiB
# pages), against the pageable staging path.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check17}
mkdir -p $OUT
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $OUT/thp.txt 2>&1
cat $OUT/thp.txt
for p in 1 2; do
  timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_p$p.log 2>&1 || exit 1
done
for f in $OUT/one_*.log; do echo "== $f"; grep -E 'seal|verify|register' $f | grep -o '"what": "[a-z_0-9]*"\|"p50_ms": [0-9.]*\|"p99_over_p50": [0-9.]*' | paste - - - ; done
