# Snappy codec on the GPU box: parity tests, then the rate lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_snappy.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_snappy.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_snappy.log | head -30; tail -3 gpurun_out/pytest_snappy.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_snappy.py ${SNAPPY_ARGS:-} > gpurun_out/bench_snappy.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_snappy.log | cut -c1-1500
exit $rc
