#!/bin/bash
# Bloom build: key words two rounds ahead (LSBM_BUILD_DEPTH=2) at 5/6/7 waves
# per SIMD, and depth 1 at 6, against the default (depth 1, 7 waves);
# the bloom GPU tests on the depth-2 library first.  Interleaved, two passes.
export TMPDIR=/tmp
OUT=gpurun_out/bloomab; mkdir -p $OUT
LSBM_LIB_PATH=$PWD/build/ab/d2w6/liblsbm_crc32c.so timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_d2w6.log 2>&1
rc=$?; echo "bloom tests (d2w6) rc=$rc"; tail -2 $OUT/pytest_d2w6.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  timeout -k 10 300 python -u tools/bench_bloom.py build --cpu-filters 0 > $OUT/base_p$p.log 2>&1 || exit 1
  for v in d2w6 d2w7 d2w5 d1w6; do
    LSBM_LIB_PATH=$PWD/build/ab/$v/liblsbm_crc32c.so timeout -k 10 300 python -u tools/bench_bloom.py build --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"ms": [0-9.]*' $f | head -1) $(grep -o '"frac": [0-9.]*' $f | head -1)"; done
