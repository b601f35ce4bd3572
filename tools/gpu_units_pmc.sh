# rocprofv3 passes over a workload (GPU box): kernel-trace stats, then one run
# per PMC counter group (never combined with trace domains).  Usage:
#   tools/gpu_units_pmc.sh <outdir> <command...>
# then `python3 tools/pmc_summary.py <outdir>` (any machine).
set -o pipefail
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- "$@" > $out/stats.log 2>&1 || { tail -20 $out/stats.log; exit 1; }
i=0
for grp in \
  "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
  "WRITE_SIZE GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
  "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $out/pmc$i -o run -- "$@" > $out/pmc$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -20 $out/pmc$i.log; exit $rc; }
done
