# Snappy over larger blocks (tools/bench_snappy.py --merge: consecutive
# db_bench blocks concatenated), after the snappy GPU tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_snappy.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_snappy.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_snappy.log; [ $rc -eq 0 ] || exit $rc
for m in ${MERGES:-1 2 3 15}; do
  timeout -k 10 300 python -u tools/bench_snappy.py --cpu-seconds 0 --reps 3 --merge $m > gpurun_out/snappy_merge$m.log 2>&1 || exit 1
  python3 - $m <<'PY'
import json, sys
m = sys.argv[1]
for l in open(f"gpurun_out/snappy_merge{m}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(m, d["metric"][:17], d["value"], d.get("sample_mismatches", d.get("roundtrip_ok")))
PY
done
