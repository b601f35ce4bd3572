#!/bin/bash
# Deferred WAL headers (the stream kernel's out[] first, each wave's header
# stores after its last row): the log GPU tests with the option on, then an
# interleaved A/B against in-place header stores (LSBM_LOG_DEFER=0).
export TMPDIR=/tmp
OUT=gpurun_out/logdefer; mkdir -p $OUT
LSBM_LOG_DEFER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stream.py tests/test_real_fixture.py -m gpu -x -q --timeout 300 --timeout-method thread -k "log or wal or stream or real" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  LSBM_LOG_DEFER=1 timeout -k 10 300 python -u tools/bench_configs.py wal > $OUT/defer_p$p.log 2>&1 || exit 1
  LSBM_LOG_DEFER=0 timeout -k 10 300 python -u tools/bench_configs.py wal > $OUT/inplace_p$p.log 2>&1 || exit 1
done
python3 tools/ab_summary.py $OUT/*_p*.log
