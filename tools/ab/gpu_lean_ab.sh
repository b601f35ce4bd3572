#!/bin/bash
# Stream kernel tests on the new library, then an interleaved A/B of the
# stream kernel against the variants under build/ab/ (LSBM_LIB_PATH) on the
# device-resident workloads of tools/bench_configs.py.
export TMPDIR=/tmp
mkdir -p gpurun_out/lean
timeout -k 10 400 python -u -m pytest tests/test_stream.py tests/test_log.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/lean/pytest_stream.log 2>&1
rc=$?; echo "stream/log tests rc=$rc"; tail -3 gpurun_out/lean/pytest_stream.log
[ $rc -eq 0 ] || exit $rc
W=${WHICH:-"wal sst4118 units4k config4"}
V=${VARIANTS:-"old"}
for pass in 1 2; do
  LSBM_RAGGED_KERNEL=stream timeout -k 10 400 python -u tools/bench_configs.py $W > gpurun_out/lean/new_p$pass.log 2>&1 || { echo "new pass $pass failed"; tail -5 gpurun_out/lean/new_p$pass.log; exit 1; }
  for v in $V; do
    LSBM_RAGGED_KERNEL=stream LSBM_LIB_PATH=$PWD/build/ab/$v/liblsbm_crc32c.so timeout -k 10 400 python -u tools/bench_configs.py $W > gpurun_out/lean/${v}_p$pass.log 2>&1 || { echo "$v pass $pass failed"; tail -5 gpurun_out/lean/${v}_p$pass.log; exit 1; }
  done
done
python3 tools/ab_summary.py gpurun_out/lean/*_p*.log
