# Snappy decoder A/B on the GPU box: parity tests of the default library, then
# interleaved bench lines: the default decoder (lane-parallel windows, paired
# copies) vs build/abl/lib_snaps.so (copies one at a time) and lib_snapw.so
# (round 2's per-tag windowed walk).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_snappy.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_snappy.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|assert" gpurun_out/pytest_snappy.log | head -30; tail -3 gpurun_out/pytest_snappy.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in ${VARIANTS:-lanes snaps snapw}; do
    if [ $v = lanes ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo "== $v pass $pass" >> gpurun_out/snappy_ab.log
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_snappy.py --cpu-seconds 0 ${SNAPPY_ARGS:-} >> gpurun_out/snappy_ab.log 2>&1 || exit 1
  done
done
grep -E "==|uncompress" gpurun_out/snappy_ab.log | cut -c1-200
