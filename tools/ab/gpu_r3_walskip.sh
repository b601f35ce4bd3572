#!/bin/bash
# Deferred WAL headers without re-reading record lengths in waves whose
# records all fit: log GPU tests, then an interleaved A/B against the
# previous library (build/ab/prevdefer); then the bloom build diagnostic.
export TMPDIR=/tmp
OUT=gpurun_out/walskip; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stream.py tests/test_real_fixture.py tests/test_log.py -m gpu -x -q --timeout 300 --timeout-method thread -k "log or wal or stream or real" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  timeout -k 10 300 python -u tools/bench_configs.py wal > $OUT/new_p$p.log 2>&1 || exit 1
  LSBM_LIB_PATH=$PWD/build/ab/prevdefer/liblsbm_crc32c.so timeout -k 10 300 python -u tools/bench_configs.py wal > $OUT/prev_p$p.log 2>&1 || exit 1
done
python3 tools/ab_summary.py $OUT/*_p*.log
bash tools/gpu_r3_bloomdiag.sh
