# PMC passes for the CRC kernel (one rocprofv3 run per counter group).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
CMD="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/pmc/p$i.log; exit $rc; }
done
