#!/bin/bash
# Round 4: GPU suite (table layer's small page-locked jobs both ways).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check15}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; grep -E "speedup=|^FAIL" $OUT/pytest_gpu.log | head; exit $rc
