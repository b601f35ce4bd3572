# Full check on the GPU box: parity tests, default bench, configs 3/4 + host-staged.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-2500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py ${CONFIGS:-config1 config3 config4 host} > gpurun_out/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' gpurun_out/configs.log
exit $rc
