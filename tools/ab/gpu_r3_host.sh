#!/bin/bash
# Host layers: their GPU tests, then the rates with phase timing, NT staging
# copy vs memcpy (LSBM_HOST_COPY=plain), then the stream kernel's event stats.
export TMPDIR=/tmp
OUT=gpurun_out/r3host
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_log.py -m gpu -x -q --timeout 300 --timeout-method thread -k "host or layer or log or table" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in nt plain nt; do
  LSBM_HOST_COPY=$v LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_$v.log 2> $OUT/timing_$v.log
  rc=$?; echo "host layers ($v) rc=$rc"; cut -c1-250 $OUT/host_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/stream_stats.sh run wal walseal units4k sst c4 > $OUT/stream_stats.log 2>&1
echo "stats rc=$?"; cat $OUT/stream_stats.log | grep -v "^W\|amdgpu.ids"
