set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cpp or level2" tests/test_multirank_gpu.py > gpurun_out/r5c1/tests.log 2>&1 && \
timeout -k 10 300 build/bench_one_table 100 4 16 > gpurun_out/r5c1/one_table.log 2> gpurun_out/r5c1/one_table.err
