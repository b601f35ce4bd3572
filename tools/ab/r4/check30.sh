#!/bin/bash
# Round 4: the bloom lookup (key_may_match) inlined into the probe kernels
# (build/abl/inl: no call, so no wait for every outstanding load at the call's
# entry; 80 / 95 VGPRs, 6 / 5 waves, no spills) against the in-tree call; and
# inlined with each probe's bit position packed 3 bits apiece (build/abl/ip:
# 69 / 83 VGPRs, 7 / 5 waves; build/abl/ip6: the filter-block probe at 6).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check30}
mkdir -p $OUT
for v in inl ip ip6; do
  LSBM_LIB_PATH=$PWD/build/abl/$v/liblsbm_crc32c.so timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bloom_$v.log 2>&1
  rc=$?; echo "bloom tests ($v) rc=$rc"; tail -1 $OUT/pytest_bloom_$v.log; [ $rc -eq 0 ] || exit $rc
done
for p in 1 2; do
  for v in default inl ip ip6; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"bench": "[a-z_]*"\|"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
