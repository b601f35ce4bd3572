# A/B of the general ragged path's longest unit (tools: build/abl/lib_u*.so built
# with -DLSBM_UNIT_ROWS=N); two interleaved passes, one process per variant.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in 1 2; do
  for v in ${VARIANTS:-base u24 u40 u48}; do
    if [ $v = base ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo -n "$v pass $pass: "
    LSBM_LIB_PATH=$L timeout -k 10 200 python3 tools/bench_configs.py config4 sst4118 --c4-blocks 4000000 --sst-blocks 524288 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['pct_hbm_peak'], d.get('sample_mismatches'), end='; ')
print()" || exit 1
  done
done
