#!/bin/bash
# Round 4: the inlined bloom lookup (in-tree) against the call (build/abl/call,
# the kernels before c5c9be4) on a second box, interleaved; then the in-tree
# bench with its CPU baseline (which runs between the GPU timings).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check31}
mkdir -p $OUT
for p in 1 2; do
  for v in default call; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
