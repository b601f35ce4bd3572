# Bloom build A/B on the GPU box: the bloom GPU tests of the default library,
# then interleaved build lines (default vs build/abl/lib_$v.so for $VARIANTS).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bloom.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_bloom.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/pytest_bloom.log | head -30; tail -3 gpurun_out/pytest_bloom.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in default ${VARIANTS:-bprev}; do
    if [ $v = default ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo "== $v pass $pass" >> gpurun_out/bloom_ab.log
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_bloom.py ${WHICH:-build} --cpu-filters 0 >> gpurun_out/bloom_ab.log 2>&1 || exit 1
  done
done
grep -E "==|bloom_" gpurun_out/bloom_ab.log | cut -c1-220
