# PMC passes over the bloom build/probe kernels (one rocprofv3 run per group).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bpmc
CMD="python3 tools/bench_bloom.py build probe --cpu-filters 0 --reps 3"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d gpurun_out/bpmc/p$i -o run -- $CMD > gpurun_out/bpmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bpmc/p$i.log; exit $rc; }
done
