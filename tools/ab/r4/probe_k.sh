#!/bin/bash
# Round 4: how the bloom kernels' time scales with k (bits per key 20, 10, 5 =
# k 13, 6, 3; filters 84, 42, 21 B): what a probe's scattered loads cost.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_probe_k}
mkdir -p $OUT
for p in 1 2; do
  for b in 20 10 5; do
    LSBM_BENCH_BPK=$b timeout -k 10 300 python -u tools/bench_bloom.py build probe block --cpu-filters 0 > $OUT/bpk${b}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
