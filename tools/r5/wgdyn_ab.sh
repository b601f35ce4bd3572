#!/bin/bash
# A/B: the fixed kernel's waves taking their workgroup's groups from an LDS
# counter (-DLSBM_WG_DYNAMIC, build/wgdyn) against the static interleave.
OUT=${OUT:-gpurun_out/r5_wgdyn}
mkdir -p $OUT
LSBM_LIB_PATH=build/wgdyn/liblsbm_crc32c.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "fixed or config5 or smoke or graph" > $OUT/test.log 2>&1 || exit 1
LSBM_LIB_PATH=build/wgdyndiag/liblsbm_crc32c.so LSBM_FIXED_SPLIT_BLOCKS=0 timeout -k 10 200 python -u tools/wave_spread.py > $OUT/spread.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/head_base_$i.log 2>&1 || exit 1
  LSBM_LIB_PATH=build/wgdyn/liblsbm_crc32c.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/head_dyn_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --blocks 10000000 --no-cpu-baseline > $OUT/s10m_base_$i.log 2>&1 || exit 1
  LSBM_LIB_PATH=build/wgdyn/liblsbm_crc32c.so timeout -k 10 200 python -u bench.py --blocks 10000000 --no-cpu-baseline > $OUT/s10m_dyn_$i.log 2>&1 || exit 1
  LSBM_LIB_PATH=build/wgdyn/liblsbm_crc32c.so LSBM_FIXED_SPLIT_BLOCKS=0 timeout -k 10 200 python -u bench.py --blocks 10000000 --no-cpu-baseline > $OUT/s10m_dyn_nosplit_$i.log 2>&1 || exit 1
done
