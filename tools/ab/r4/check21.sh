#!/bin/bash
# Round 4: staged small jobs with doubling chunks (in-tree) against equal
# chunks (LSBM_CHUNK_RAMP=0); pageable seals staged too (LSBM_AUTO_LOCK=0).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check21}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "table or sst or seal or pinned" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2 3; do
  for v in geo equal; do
    if [ $v = geo ]; then R=1; else R=0; fi
    LSBM_AUTO_LOCK=0 LSBM_CHUNK_RAMP=$R timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/one_*.log; do echo "$(basename $f) $(grep -E '"(seal|verify)_pageable"' $f | grep -o '"p50_ms": [0-9.]*' | paste -sd' ')"; done
LSBM_AUTO_LOCK=0 LSBM_HOST_TIMING=1 timeout -k 10 120 build/bench_one_table 20 4 > $OUT/one_geo_timing.log 2>&1; echo "timing rc=$?"
