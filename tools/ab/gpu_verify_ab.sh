# SSTable / WAL verify A/B: the parity tests of the default library, then
# interleaved `tools/bench_configs.py sst4118 wal` lines: default vs build/abl/lib_$v.so.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_log.py tests/test_real_fixture.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_verify.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_verify.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in default ${VARIANTS:-v2}; do
    if [ $v = default ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo "== $v pass $pass" >> gpurun_out/verify_ab.log
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_configs.py sst4118 wal >> gpurun_out/verify_ab.log 2>&1 || exit 1
  done
done
