#!/bin/bash
# Round 4: the WAL seal's header stores per chunk as chunks complete (in-tree)
# against all of them after the last chunk (LSBM_LOG_POST_AFTER=1).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check23}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_log.py tests/test_gpu_parity.py -m gpu -x -q -k "log or wal or table_layer" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in chunk after; do
    if [ $v = after ]; then export LSBM_LOG_POST_AFTER=1; else unset LSBM_LOG_POST_AFTER; fi
    timeout -k 10 300 build/bench_host_layers 200 1024 > $OUT/host_${v}_p$p.log 2>&1 || exit 1
  done
done
unset LSBM_LOG_POST_AFTER
for f in $OUT/host_*.log; do echo "$(basename $f) $(grep -o '"what": "wal".*"verify_GBps": [0-9.]*' $f | grep -o '"seal_GBps": [0-9.]*\|"verify_GBps": [0-9.]*' | paste -sd' ')"; done
