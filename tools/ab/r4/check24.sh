#!/bin/bash
# Round 4: filter-block lookups pipelined ahead of the keys (in-tree) against
# one after another behind the hash (build/abl/noahead); bloom tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check24}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom.log 2>&1
rc=$?; echo "bloom tests rc=$rc"; tail -1 $OUT/pytest_bloom.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default noahead; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
