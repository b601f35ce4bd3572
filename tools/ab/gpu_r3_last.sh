#!/bin/bash
# Last rehearsal on the final library: every GPU test, smoke(), the default
# bench, the WAL configs and the WAL PMC of the stream kernel (and units).
export TMPDIR=/tmp
bash tools/gpu_final.sh || exit $?
OUT=gpurun_out/last; mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_configs.py wal config4 sst4118 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; python3 tools/ab_summary.py $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof
WHICH=wal bash tools/gpu_prof_ragged.sh > $OUT/prof_wal.log 2>&1; echo "prof rc=$?"
