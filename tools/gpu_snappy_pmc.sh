# Kernel-trace stats and PMC passes over the snappy kernels (one rocprofv3 run per group).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/spmc
CMD="python3 tools/bench_snappy.py --reps 3 --cpu-seconds 0"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/spmc/stats -o run -- $CMD > gpurun_out/spmc/stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/spmc/stats.log; exit $rc; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d gpurun_out/spmc/p$i -o run -- $CMD > gpurun_out/spmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/spmc/p$i.log; exit $rc; }
done
