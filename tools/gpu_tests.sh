# GPU parity tests only (optionally a subset: TESTS="tests/test_log.py").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -3 gpurun_out/pytest_gpu.log
exit $rc
