#!/bin/bash
# Every device entry point of the path under rocprofv3 (round 5): per entry, a
# --kernel-trace --stats pass (average kernel duration from rocprof) and a
# separate --pmc FETCH_SIZE pass (HBM read bytes, gfx950 x2 correction), then
# tools/roofline_summary.py joins them with the entry's algorithmic bytes.
# The per-dispatch counter CSVs are summarised and deleted as they go (gpurun
# copies back at most 64 MiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/roofline}
mkdir -p $OUT
ENTRIES=${ENTRIES:-"fixed4k config3 config4 sst_ext sst_seal sst_crcs sst_verify log_seal log_crcs log_verify"}
for e in $ENTRIES; do
  mkdir -p $OUT/$e
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$e/stats -o run -- \
    python3 tools/roofline_all.py $e > $OUT/$e/stats.log 2>&1
  rc=$?; echo "$e stats rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$e/stats.log; exit $rc; }
  LSBM_SPIN_S=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$e/pmc -o run -- \
    python3 tools/roofline_all.py $e --reps 5 > $OUT/$e/pmc.log 2>&1
  rc=$?; echo "$e pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$e/pmc.log; exit $rc; }
  python3 tools/roofline_summary.py $OUT $e || exit 1
  rm -f $OUT/$e/pmc/run_counter_collection.csv
  [ -n "$KEEP_TRACE" ] || rm -f $OUT/$e/stats/run_kernel_trace.csv
done
python3 tools/roofline_summary.py $OUT
