#!/bin/bash
# Round-3 check: every GPU test, smoke, the default bench, the ragged configs
# (default kernel policy), the host layers with phase timing, and their trace.
export TMPDIR=/tmp
OUT=gpurun_out/r3check
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py wal sst4118 config4 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; python3 tools/ab_summary.py $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2> $OUT/host_timing.log
rc=$?; echo "host layers rc=$rc"; cut -c1-400 $OUT/host_layers.log; [ $rc -eq 0 ] || exit $rc
python3 - $OUT/host_timing.log <<'PY'
import collections, json, sys
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
for l in open(sys.argv[1]):
    if l.startswith('{"host_timing"'):
        d = json.loads(l); a = agg[d["host_timing"]]
        a[0] += 1; a[1] += d["total_ms"]; a[2] += d["copy_ms"]; a[3] += d["wait_ms"]; a[4] += d["post_ms"]
for k, a in agg.items():
    print(f"{k:22s} calls={a[0]:5d} total={a[1]:9.1f} ms copy={a[2]:9.1f} wait={a[3]:9.1f} post={a[4]:8.1f}")
PY
OUT=$OUT/host_trace bash tools/gpu_host_trace.sh
