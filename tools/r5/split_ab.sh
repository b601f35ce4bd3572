#!/bin/bash
# Launch-split A/Bs: the ragged split on the parity
# tests (tiny split size so every batch splits), then config 4 with ragged
# launches of 0 / 1M / 2M blocks, config 3 with fixed launches of 0 / 64K /
# 256K blocks, and the headline with 1M (one launch) / 512K / 256K.
OUT=${OUT:-gpurun_out/r5_rsplit}
mkdir -p $OUT
LSBM_RAGGED_SPLIT_BLOCKS=1000 timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "ragged or batch or stream or offsets" > $OUT/test_split1000.log 2>&1 || exit 1
for i in 1 2; do
  for s in 0 1048576 2097152; do
    LSBM_RAGGED_SPLIT_BLOCKS=$s timeout -k 10 200 python -u tools/bench_configs.py config4 > $OUT/c4_${s}_$i.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for s in 0 65536 262144; do
    LSBM_FIXED_SPLIT_BLOCKS=$s timeout -k 10 200 python -u tools/bench_configs.py config3 > $OUT/c3_${s}_$i.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for s in 1048576 524288 262144; do
    LSBM_FIXED_SPLIT_BLOCKS=$s timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/head_${s}_$i.log 2>&1 || exit 1
  done
done
