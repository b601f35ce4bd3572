#!/bin/bash
# Rehearsal of the driver's round end (GPU suite, smoke(), the
# default bench), then the host-layer CPU-budget bench, the bloom line and the
# headline kernel's rocprofv3 stats + PMC passes (tools/gpu_profile.sh).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
# the per-GPU rate on one config-5 shard (10M blocks: what each rank of the N > 1 runs checksums)
timeout -k 10 300 python -u bench.py --blocks 10000000 --no-cpu-baseline > $OUT/bench_10m.log 2>&1
rc=$?; echo "bench_10m rc=$rc"; tail -1 $OUT/bench_10m.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_one_table 100 4 > $OUT/one_table.log 2>&1
rc=$?; echo "one_table rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2>&1
rc=$?; echo "host_layers rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_bloom.py > $OUT/bench_bloom.log 2>&1
rc=$?; echo "bloom rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh $OUT/profile
rc=$?; echo "profile rc=$rc"; du -sh $OUT; exit $rc
