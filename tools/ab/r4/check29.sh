#!/bin/bash
# Round 4: bloom lookups with each probe's bit position packed 3 bits apiece
# into two registers instead of 16 mask registers (then in-tree, now reverted: the one-filter
# probe at 70 VGPRs, 7 waves per SIMD; the filter-block probe at 84, 5 waves)
# against the kernels before (build/abl/r4head) and the filter-block probe held
# to 6 waves (build/abl/b6, 80 VGPRs, 2 spilled).  Bloom tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check29}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom.log 2>&1
rc=$?; echo "bloom tests rc=$rc"; tail -1 $OUT/pytest_bloom.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default r4head b6; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
