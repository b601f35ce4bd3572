# Host-layer A/B on one box: SealTables with and without its host trailer
# writes (LSBM_DIAG_SEAL_NO_WRITE: a temporary diagnostic build, not in the product).
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in 1 2; do
  for v in base nowrite; do
    echo "== $v pass $pass" >> gpurun_out/host_ab.log
    if [ $v = nowrite ]; then E="LSBM_DIAG_SEAL_NO_WRITE=1"; else E="LSBM_X=0"; fi
    env $E timeout -k 10 300 build/bench_host_layers ${TABLES:-1000} 64 >> gpurun_out/host_ab.log 2>&1 || exit 1
  done
done
grep -E "==|compaction" gpurun_out/host_ab.log | cut -c1-260
