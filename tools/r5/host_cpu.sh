# Host-layer rates with host CPU per call / table / GB (round 5), two passes,
# then the compaction three ways (reference, Level-1 relink, GPU ends).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_host2; mkdir -p $O
for p in 1 2; do
  timeout -k 10 300 build/bench_host_layers 1000 1024 > $O/host_layers_p$p.log 2>&1 || exit 1
  LSBM_AUTO_LOCK=0 timeout -k 10 300 build/bench_host_layers 1000 1024 > $O/host_layers_nolock_p$p.log 2>&1 || exit 1
done
for b in gpu_compaction gpu_compaction_l1; do timeout -k 10 300 oracle/_ref/$b 4 16 16 >> $O/compaction.log 2>&1 || exit 1; done
