#!/bin/bash
# Round 4, verdict item 1: the one-table seal stall.  Per-call distributions
# and cgroup throttling (build/bench_one_table), the same with per-call phase
# timing, then a kernel + memory-copy + HIP-runtime trace of the calls.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_one_table}
mkdir -p $OUT
{ cat /sys/fs/cgroup/cpu.max; nproc; cat /sys/devices/system/node/online;
  for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done;
  for d in /sys/bus/pci/devices/*; do v=$(cat $d/vendor); c=$(cat $d/class);
    if [ "$v" = 0x1002 ] && [ "${c:0:4}" = 0x12 ]; then echo "gpu $(basename $d) numa $(cat $d/numa_node)"; fi; done;
  taskset -p $$; } > $OUT/box.txt 2>&1
cat $OUT/box.txt
timeout -k 10 180 build/bench_one_table ${REPS:-100} 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; cat $OUT/one_table.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 180 build/bench_one_table ${REPS:-100} 4 > $OUT/one_table_timing.log 2> $OUT/timing.log
rc=$?; echo "one_table timing rc=$rc"; cut -c1-220 $OUT/one_table_timing.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d $OUT/trace -o run -- build/bench_one_table ${REPS:-100} 1 > $OUT/trace_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; grep '"what"' $OUT/trace_bench.log | cut -c1-220
ls -la $OUT/trace/* | head
exit $rc
