#!/bin/bash
# Round 4: the DMA path's floor for one page-locked 16 MiB table (raw DMA from
# the registered image / a hipHostMalloc'd copy, whole / 4 chunks, + verify).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check10}
mkdir -p $OUT
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-260 $OUT/one_table.log | grep -E "locked|dma"; [ $rc -eq 0 ] || exit $rc
LSBM_ZERO_COPY_MAX_MB=0 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_dma.log 2>&1
rc=$?; echo "one_table dma rc=$rc"; cut -c1-260 $OUT/one_table_dma.log | grep -E "locked|dma"; exit $rc
