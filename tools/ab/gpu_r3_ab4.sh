#!/bin/bash
export TMPDIR=/tmp
VARIANTS="nopre v3" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh || exit $?
OUT=gpurun_out/r3host4; mkdir -p $OUT
LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host.log 2> $OUT/timing.log
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host.log; grep -v Tables $OUT/timing.log; [ $rc -eq 0 ] || exit $rc
WHICH=wal bash tools/gpu_prof_ragged.sh > gpurun_out/prof_wal.log 2>&1; echo "prof rc=$?"; tail -12 gpurun_out/prof_wal.log
