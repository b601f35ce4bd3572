#!/bin/bash
# Round-3 rehearsal, part A: every GPU test, smoke(), the default bench, then
# the headline profile (rocprof stats + PMC passes -> profiles/traffic.json).
export TMPDIR=/tmp
OUT=gpurun_out/finalA
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh $OUT/profile > $OUT/profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -3 $OUT/profile.log; exit $rc
