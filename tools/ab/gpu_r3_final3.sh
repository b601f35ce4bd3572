#!/bin/bash
# Rehearsal on the library with the per-wave seal merges and deferred WAL
# headers: every GPU test, smoke(), the default bench, then the configs.
export TMPDIR=/tmp
bash tools/gpu_final.sh || exit $?
OUT=gpurun_out/final3; mkdir -p $OUT
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.log $OUT/
timeout -k 10 400 python -u tools/bench_configs.py wal config4 sst4118 config1 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; python3 tools/ab_summary.py $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
