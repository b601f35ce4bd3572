#!/bin/bash
# Round 4: GPU suite on the new host runtime + per-window stream fallback,
# WAL / config-4 rates (in order, length-sorted, shuffled), the one-table
# distributions (plain, after a 300 ms pause, with phase timing) and the
# compaction / WAL host-layer rates.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check4}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py wal config4 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; cut -c1-1500 $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-330 $OUT/one_table.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 16 300 > $OUT/one_table_idle.log 2>&1
rc=$?; echo "one_table idle rc=$rc"; cut -c1-330 $OUT/one_table_idle.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 180 build/bench_one_table 50 4 > $OUT/one_table_timing.log 2> $OUT/timing.log
rc=$?; echo "one_table timing rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; exit $rc
