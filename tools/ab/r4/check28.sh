#!/bin/bash
# Round 4: bloom probes with each round's lookups tested during the next round
# (tools/ab/r4/probe_defer.patch, 4 waves per SIMD) against testing them at once (build/abl/nodefer,
# the kernels before: 6 / 5 waves) and deferred at 5 waves with spills
# (build/abl/d5).  Bloom tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check28}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom.log 2>&1
rc=$?; echo "bloom tests rc=$rc"; tail -1 $OUT/pytest_bloom.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default nodefer d5; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*\|"no_false_negatives": [a-z]*' $f | paste -sd' ')"; done
