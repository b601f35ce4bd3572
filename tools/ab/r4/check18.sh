#!/bin/bash
# Round 4: small jobs' pageable images page-locked per call (CallLocks):
# GPU suite, one table per call (default vs LSBM_AUTO_LOCK=0), host layers.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check18}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=|^FAIL" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in auto staged; do
    if [ $v = auto ]; then A=1; else A=0; fi
    LSBM_AUTO_LOCK=$A timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/one_*.log; do echo "== $f"; grep -E '"(seal|verify)_(pageable|locked)"|concurrent_seal|alternate' $f | grep -o '"what": "[a-z_0-9]*"\|"p50_ms": [0-9.]*\|"p99_over_p50": [0-9.]*\|"max_ms": [0-9.]*\|"concurrent_GBps": [0-9.]*' | paste -sd' ' | cut -c1-600; done
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-250 $OUT/host_layers.log; exit $rc
