#!/bin/bash
# Round 4: GPU suite; WAL / config-4 rates (stream kernel's early order check);
# one-table with zero copy (default) and with DMA chunks on the copy stream;
# host layers; bloom (build without the binary search).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check9}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py wal config4 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; cut -c1-1500 $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-330 $OUT/one_table.log; [ $rc -eq 0 ] || exit $rc
LSBM_ZERO_COPY_MAX_MB=0 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_dma.log 2>&1
rc=$?; echo "one_table dma rc=$rc"; cut -c1-330 $OUT/one_table_dma.log | grep locked; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/bench_bloom.py > $OUT/bench_bloom.log 2>&1
rc=$?; echo "bloom rc=$rc"; grep '^{' $OUT/bench_bloom.log | cut -c1-300; exit $rc
