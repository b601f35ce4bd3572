#!/bin/bash
# Round 4: the bloom probes with and without their filter round trip
# (build/abl/nofl: LSBM_DIAG_NO_FILTER_LOADS, wrong answers): how much of a
# probe round is the exposed k-byte + probe-byte latency.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_probe_nofl}
mkdir -p $OUT
for p in 1 2; do
  for v in default nofl; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
