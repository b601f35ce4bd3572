# Bloom bench + kernel-trace stats on the GPU box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/bench_bloom.py > gpurun_out/bloom.log 2>&1
rc=$?; echo "bloom rc=$rc"; grep '^{' gpurun_out/bloom.log | cut -c1-600; [ $rc -eq 0 ] || { tail -20 gpurun_out/bloom.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bloomprof -o run -- python3 tools/bench_bloom.py --cpu-filters 0 --reps 10 > gpurun_out/bloomprof.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -d, -f1-4 gpurun_out/bloomprof/run_kernel_stats.csv | cut -c1-200
exit $rc
