#!/bin/bash
# Round 4: GPU suite (the zero-copy seal now stores its trailers in place over
# PCIe); bloom probe with the filter handle one round ahead (in-tree, 6 waves,
# 32 B spill; ha5: 5 waves) against the in-tree probe; one table:
# zero copy (in place), zero copy posted by the host, DMA chunks, and the DMA
# path's floor.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check11}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in default nofast fast5 ha6; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py probe block --cpu-filters 0 > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
done
for p in 1 2; do
  for v in default nofold; do
    if [ $v = default ]; then L=""; else L="$PWD/build/abl/$v/liblsbm_crc32c.so"; fi
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py build --cpu-filters 0 > $OUT/build_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/*_p*.log; do echo "$(basename $f) $(grep -o '"ms": [0-9.]*\|"frac": [0-9.]*' $f | paste -sd' ')"; done
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-230 $OUT/one_table.log | grep -E "locked|dma|host_copy"; [ $rc -eq 0 ] || exit $rc
LSBM_ZERO_COPY_SEAL_POST=1 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_post.log 2>&1
rc=$?; echo "one_table post rc=$rc"; cut -c1-230 $OUT/one_table_post.log | grep -E "_locked"; [ $rc -eq 0 ] || exit $rc
LSBM_ZERO_COPY_MAX_MB=0 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table_dma.log 2>&1
rc=$?; echo "one_table dma rc=$rc"; cut -c1-230 $OUT/one_table_dma.log | grep -E "_locked"; exit $rc
