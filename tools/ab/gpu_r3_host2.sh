#!/bin/bash
# Host layers after the WAL changes: their GPU tests, then the rates (twice).
export TMPDIR=/tmp
OUT=gpurun_out/r3host3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_log.py tests/test_real_fixture.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_p$p.log 2> $OUT/timing_p$p.log
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_p$p.log; grep -v Tables $OUT/timing_p$p.log; [ $rc -eq 0 ] || exit $rc
done
