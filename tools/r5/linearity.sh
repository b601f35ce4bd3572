# Full-size linearity checks (configs 2 and 3; config 5's shards through bench.py --gpus 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_parity.py -k "config2_full or config3_full" > $O/tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_multirank_gpu.py >> $O/tests.log 2>&1
