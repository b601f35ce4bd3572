#!/bin/bash
# Round 4: bloom rounds with each key's (start, length) computed once and
# carried, single-compare wave masks, the filter count carried between rounds
# (in-tree; now also two register sets alternating between rounds and scalar
# span tests) against the previous kernels (build/abl/r4base); bloom tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check26}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom.log 2>&1
rc=$?; echo "bloom tests rc=$rc"; tail -1 $OUT/pytest_bloom.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default r4base; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py build probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
