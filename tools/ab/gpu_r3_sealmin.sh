#!/bin/bash
# Small-batch SST seal: config 1's 45K blocks one pass in place (default,
# below 131,072 blocks) vs dense CRCs + per-wave trailer merges
# (LSBM_SEAL_MIN_BLOCKS=1), interleaved.
export TMPDIR=/tmp
OUT=gpurun_out/sealmin; mkdir -p $OUT
LSBM_SEAL_MIN_BLOCKS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sst or seal" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2 3; do
  LSBM_SEAL_MIN_BLOCKS=1 timeout -k 10 300 python -u tools/bench_configs.py config1 > $OUT/fused_p$p.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/bench_configs.py config1 > $OUT/onepass_p$p.log 2>&1 || exit 1
done
grep -H -o '"gpu_ms": {[^}]*}' $OUT/*_p*.log
