#!/bin/bash
# Kernel + memory-copy timeline of the C++ host layers (SealTables vs
# VerifyTables on the same pageable and page-locked images, the WAL group
# commit and its verify), then tools/host_timeline.py's per-phase summary.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/host_trace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- \
  build/bench_host_layers ${TABLES:-250} ${WAL_MB:-512} > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; cut -c1-300 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
python3 tools/host_timeline.py $OUT/trace > $OUT/timeline.txt 2>&1; cat $OUT/timeline.txt
