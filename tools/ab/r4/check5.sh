#!/bin/bash
# Round 4: GPU suite; WAL / config-4 rates (in order, length-sorted, shuffled);
# one-table distributions; host layers; bloom rates (cheaper probe sequence)
# and the FETCH_SIZE calibration for small scattered reads.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check5}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py wal config4 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; cut -c1-1500 $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cut -c1-330 $OUT/one_table.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 180 build/bench_one_table 50 4 > $OUT/one_table_timing.log 2> $OUT/timing.log
rc=$?; echo "one_table timing rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/bench_bloom.py > $OUT/bench_bloom.log 2>&1
rc=$?; echo "bloom rc=$rc"; grep '^{' $OUT/bench_bloom.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $grp | cut -c1-5)
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $OUT/calib_$n -o run -- build/fetch_calib > $OUT/calib_$n.log 2>&1
  rc=$?; echo "calib $n rc=$rc"; cat $OUT/calib_$n.log | grep pattern; [ $rc -eq 0 ] || exit $rc
done
exit 0
