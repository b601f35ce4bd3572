# Run the ragged-path GPU tests against the bounds-checked debug library
# (build/dbg, -DLSBM_DEBUG_BOUNDS): wild accesses are printed and skipped.
set -o pipefail
mkdir -p gpurun_out
cp lsbm_amd/liblsbm_crc32c.so gpurun_out/product.so
cp build/dbg/liblsbm_crc32c.so lsbm_amd/liblsbm_crc32c.so
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -m pytest -x -q -s tests/test_gpu_parity.py -k "(general_geometry or ragged or verify or sst or host_staged or config2) and not cpp" > gpurun_out/dbg_tests.log 2>&1
rc=$?
grep -E "OOB|passed|failed|Error" | grep -v "^units:" gpurun_out/dbg_tests.log | head -40
cp gpurun_out/product.so lsbm_amd/liblsbm_crc32c.so
exit $rc
