#!/bin/bash
export TMPDIR=/tmp
VARIANTS="noearly nomerge2" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh || exit $?
bash tools/stream_stats.sh run wal > gpurun_out/stream_stats_ab7.log 2>&1; grep "wal wave" gpurun_out/stream_stats_ab7.log
