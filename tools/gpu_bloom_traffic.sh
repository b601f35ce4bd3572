#!/bin/bash
# HBM traffic of the three bloom kernels (build, probe, filter-block probe):
# one rocprofv3 --pmc pass each for FETCH_SIZE and WRITE_SIZE (they do not fit
# one pass), then tools/bloom_traffic.py -> profiles/bloom_traffic.json, which
# tools/bench_bloom.py puts into its lines' roofline.traffic.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/bloom_traffic}
mkdir -p $OUT
CMD="python3 tools/bench_bloom.py build probe block --cpu-filters 0 --reps 3"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/bloom_traffic.py $OUT && cp profiles/bloom_traffic.json $OUT/
