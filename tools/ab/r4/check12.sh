#!/bin/bash
# Round 4: worker pool with atomic piece claims; small page-locked jobs as one
# whole-image DMA + kernel per table (default) vs zero copy (LSBM_SMALL_LOCKED=zc)
# vs the chunk pipeline; host layers at full size.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check12}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-230 $OUT/one_table.log | grep -E "seal|verify|host_copy|concurrent"; [ $rc -eq 0 ] || exit $rc
LSBM_SMALL_LOCKED=zc timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_zc.log 2>&1
rc=$?; echo "one_table zc rc=$rc"; cut -c1-230 $OUT/one_table_zc.log | grep -E "_locked|host_copy"; [ $rc -eq 0 ] || exit $rc
LSBM_ZERO_COPY_MAX_MB=0 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_chunks.log 2>&1
rc=$?; echo "one_table chunks rc=$rc"; cut -c1-230 $OUT/one_table_chunks.log | grep -E "_locked"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; exit $rc
