#!/bin/bash
# Round 4: occupancy of the inlined-lookup probes -- the filter-block probe
# held to 6 waves per SIMD (build/abl/b6s: 80 VGPRs, 15 spilled) and the
# one-filter probe allowed 5 (build/abl/p5: 86 VGPRs) against in-tree (6 / 5).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check32}
mkdir -p $OUT
for p in 1 2; do
  for v in default b6s p5; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
