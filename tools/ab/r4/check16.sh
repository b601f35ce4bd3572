#!/bin/bash
# Round 4: the table pipeline's short first chunk (in-tree) against equal
# chunks (LSBM_CHUNK_RAMP=0), one table per call, interleaved, two passes;
# the table-layer GPU tests first.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check16}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "table or sst or seal or pinned" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in ramp equal; do
    if [ $v = ramp ]; then R=1; else R=0; fi
    LSBM_CHUNK_RAMP=$R timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/one_*.log; do echo "== $f"; grep -E '"(seal|verify)_(pageable|locked)"|concurrent_seal|register' $f | grep -o '"what": "[a-z_]*"\|"p50_ms": [0-9.]*\|"p99_over_p50": [0-9.]*\|"concurrent_GBps": [0-9.]*' | paste -sd' '; done
LSBM_HOST_TIMING=1 timeout -k 10 120 build/bench_one_table 20 4 > $OUT/one_timing.log 2>&1; echo "timing rc=$?"
