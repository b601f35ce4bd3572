#!/bin/bash
# The stream kernel's log test first (alone), then the whole GPU suite.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stream.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k log_records > gpurun_out/pytest_stream_log.log 2>&1
rc=$?
echo "log test rc=$rc"; tail -3 gpurun_out/pytest_stream_log.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -30; tail -3 gpurun_out/pytest_gpu.log
exit $rc
