# Round profile of the headline kernel (run on the GPU box from the repo root):
#   kernel-trace stats, then separate --pmc passes (gfx950 slot limits), then
#   tools/traffic.py turns them into profiles/traffic.json for bench.py.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/profile}
mkdir -p $OUT
# the stats pass runs exactly the driver's default bench command
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py > $OUT/stats.log 2>&1 || exit $?
CMD="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
i=0
for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $OUT/pmc$i -o run -- $CMD > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $OUT && cp profiles/traffic.json $OUT/
grep "^{\"metric" $OUT/stats.log > $OUT/stats_bench_line.json
