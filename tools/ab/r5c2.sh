set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gpu_sealed_table_builder" > $O/tests.log 2>&1 && \
bash tools/gpu_units_pmc.sh $O/wal_pmc python3 tools/bench_configs.py wal > $O/wal_pmc.log 2>&1 && \
python3 tools/pmc_summary.py $O/wal_pmc > $O/wal_pmc_summary.txt 2>&1
rc=$?
# (the per-dispatch counter CSVs exceed gpurun's 64 MiB copy-back: keep the summary)
rm -rf $O/wal_pmc/pmc*/ $O/wal_pmc/stats/*trace*
du -sh $O
exit $rc
