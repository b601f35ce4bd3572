#!/bin/bash
# Config 1 with lsbm's own db_bench on the GPU box: the Level-2 parity test
# (tests/test_gpu_parity.py::test_db_bench_gpu_tables), then the three builds
# interleaved (tools/db_bench_ab.py).  Output under gpurun_out/dbbench/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dbbench; mkdir -p $OUT
nproc > $OUT/host.txt; lscpu | grep "Model name" >> $OUT/host.txt
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  tests/test_gpu_parity.py -k db_bench_gpu > $OUT/test.log 2>&1 || { echo "test failed"; tail -30 $OUT/test.log; exit 1; }
timeout -k 10 600 python -u tools/db_bench_ab.py --passes ${PASSES:-5} > $OUT/ab.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
# the same at 10M writes (a run long enough that the GPU's one-time start-up is amortised)
timeout -k 10 800 python -u tools/db_bench_ab.py --passes 3 --writes 10000000 > $OUT/ab_10m.log 2>&1 || { echo "ab 10m failed"; tail -20 $OUT/ab_10m.log; exit 1; }
tail -1 $OUT/ab_10m.log
