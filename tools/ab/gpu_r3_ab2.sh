#!/bin/bash
# Stream kernel A/B (in-tree vs build/ab variants, every eligible batch on the
# stream kernel), then the host layers.
export TMPDIR=/tmp
VARIANTS="v3 v4s2" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh || exit $?
OUT=gpurun_out/r3host2
mkdir -p $OUT
LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host.log 2> $OUT/timing.log
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host.log; exit $rc
