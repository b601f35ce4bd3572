#!/bin/bash
# Round 4: big page-locked jobs' chunk DMAs on the stages' streams (in-tree)
# against one copy stream (LSBM_DIRECT_COPY_STREAM=1): host layers, two passes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check20}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "table or sst or seal or pinned" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  for v in stage copy; do
    if [ $v = copy ]; then export LSBM_DIRECT_COPY_STREAM=1; else unset LSBM_DIRECT_COPY_STREAM; fi
    timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_${v}_p$p.log 2>&1 || exit 1
  done
done
unset LSBM_DIRECT_COPY_STREAM
for f in $OUT/host_*.log; do echo "== $f"; grep -o '"pinned": [01], "seal": "OK", "seal_s": [0-9.]*, "seal_GBps": [0-9.]*, "verify": "OK", "verify_s": [0-9.]*, "verify_GBps": [0-9.]*' $f; done
