# General ragged path: longest unit 48 (default) vs 96 / 128 rows
# (build/abl/lib_u<N>.so, -DLSBM_UNIT_ROWS=N) on config 4, its lengths sorted
# (c4sorted) and equal blocks of its mean length (c4uniform); two passes.
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in 1 2; do
  for v in ${VARIANTS:-u48 u96 u128}; do
    if [ $v = u48 ]; then L=""; else L="build/abl/lib_$v.so"; fi
    echo "== $v pass $pass" >> gpurun_out/units_rows_ab.log
    LSBM_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_configs.py config4 c4sorted c4uniform >> gpurun_out/units_rows_ab.log 2>&1 || exit 1
  done
done
grep -E "==|pct_hbm" gpurun_out/units_rows_ab.log | sed 's/"payload_GiB.*"ms"/"ms"/' | cut -c1-160
