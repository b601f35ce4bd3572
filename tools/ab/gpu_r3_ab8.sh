#!/bin/bash
export TMPDIR=/tmp
LSBM_LIB_PATH=$PWD/build/ab/s2fifo/liblsbm_crc32c.so timeout -k 10 400 python -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s2fifo.log 2>&1
rc=$?; echo "s2fifo stream tests rc=$rc"; tail -1 gpurun_out/pytest_s2fifo.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="s2fifo" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh
