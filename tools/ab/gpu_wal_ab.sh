# WAL A/B: the log GPU tests of the default library, then interleaved
# `tools/bench_configs.py wal` lines: default vs build/abl/lib_$v.so.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_log.py tests/test_real_fixture.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_log.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_log.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in default ${VARIANTS:-lb}; do
    if [ $v = default ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo "== $v pass $pass" >> gpurun_out/wal_ab.log
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_configs.py wal >> gpurun_out/wal_ab.log 2>&1 || exit 1
  done
done
