#!/bin/bash
# Diagnostic: the bloom build without its k LDS probe writes per key
# (wrong filters; timing only) against the product build, interleaved.
export TMPDIR=/tmp
OUT=gpurun_out/bloomdiag; mkdir -p $OUT
for p in 1 2; do
  timeout -k 10 300 python -u tools/bench_bloom.py build --cpu-filters 0 > $OUT/base_p$p.log 2>&1 || exit 1
  LSBM_LIB_PATH=$PWD/build/ab/nowr/liblsbm_crc32c.so timeout -k 10 300 python -u tools/bench_bloom.py build --cpu-filters 0 > $OUT/nowr_p$p.log 2>&1
  echo "nowr pass $p rc=$?"
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"ms": [0-9.]*' $f | head -1) $(grep -o '"frac": [0-9.]*' $f | head -1)"; done
