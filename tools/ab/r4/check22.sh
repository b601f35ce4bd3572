#!/bin/bash
# Round 4: lock-free worker pool (job slots + hazard pointers): pool overhead,
# GPU suite, staged one-table calls (doubling chunks vs equal), host layers.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check22}
mkdir -p $OUT
timeout -k 10 120 python3 tools/ab/r4/pool_overhead.py > $OUT/pool_overhead.log 2>&1 || exit 1
cat $OUT/pool_overhead.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; grep -E "speedup=|^FAIL" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in geo equal; do
    if [ $v = geo ]; then R=1; else R=0; fi
    LSBM_AUTO_LOCK=0 LSBM_CHUNK_RAMP=$R timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/one_*.log; do echo "$(basename $f) $(grep -E '"(seal|verify)_pageable"|host_copy' $f | grep -o '"what": "[a-z_0-9A-Z]*"\|"p50_ms": [0-9.]*' | paste -sd' ')"; done
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-250 $OUT/host_layers.log; exit $rc
