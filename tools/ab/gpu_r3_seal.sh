#!/bin/bash
# The fused seal (trailers merged in the units kernel's wave epilogue): its
# GPU tests, then an interleaved A/B against round 2's separate scatter pass
# (LSBM_SEAL_SCATTER=1) on 1M x 4,118-B blocks.
export TMPDIR=/tmp
OUT=gpurun_out/seal; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_real_fixture.py tests/test_ref_link.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sst or seal or table or real or link" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 1 2; do
  timeout -k 10 300 python -u tools/bench_configs.py sst4118 > $OUT/fused_p$p.log 2>&1 || exit 1
  LSBM_SEAL_SCATTER=1 timeout -k 10 300 python -u tools/bench_configs.py sst4118 > $OUT/scatter_p$p.log 2>&1 || exit 1
done
python3 tools/ab_summary.py $OUT/*_p*.log
