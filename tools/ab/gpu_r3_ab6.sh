#!/bin/bash
# kBank A/B (rows per load bank: 3 in-tree, 4 and 5 as variants); the
# variants' own stream / log tests first (the general row's bank select).
export TMPDIR=/tmp
for v in b4 b5; do
  LSBM_LIB_PATH=$PWD/build/ab/$v/liblsbm_crc32c.so timeout -k 10 400 python -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "$v stream tests rc=$rc"; tail -1 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="b4 b5" WHICH="wal units4k config4 sst4118" bash tools/gpu_lean_ab.sh
