#!/bin/bash
# Round 4 rehearsal of the driver's round end: GPU suite, smoke(), the default
# bench; then the headline kernel's rocprofv3 stats and PMC passes
# (tools/gpu_profile.sh) into gpurun_out/r4_final/profile.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh $OUT/profile
rc=$?; echo "profile rc=$rc"; exit $rc
