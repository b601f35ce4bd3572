#!/bin/bash
# Round 4: the host runtime (sessions per caller, NUMA-local staging, the
# concurrent pool, equal chunks, 4 stages): the full GPU suite, then the
# one-table distributions (plain, after a 300 ms idle pause, with phase
# timing) and the compaction / WAL host-layer rates.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_host2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-330 $OUT/one_table.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 16 300 > $OUT/one_table_idle.log 2>&1
rc=$?; echo "one_table idle rc=$rc"; cut -c1-330 $OUT/one_table_idle.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 180 build/bench_one_table 50 4 > $OUT/one_table_timing.log 2> $OUT/timing.log
rc=$?; echo "one_table timing rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; exit $rc
