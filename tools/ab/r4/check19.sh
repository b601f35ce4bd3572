#!/bin/bash
# Round 4: per-call page locks, phase order (verify first) and timing.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check19}
mkdir -p $OUT
LSBM_BENCH_VERIFY_FIRST=1 timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_vfirst.log 2>&1 || exit 1
LSBM_HOST_TIMING=1 LSBM_BENCH_VERIFY_FIRST=1 timeout -k 10 180 build/bench_one_table 30 4 > $OUT/one_vfirst_timing.log 2>&1 || exit 1
grep -E '"(seal|verify|verify_again)_(pageable|locked)"|alternate' $OUT/one_vfirst.log | grep -o '"what": "[a-z_0-9]*"\|"p50_ms": [0-9.]*\|"max_ms": [0-9.]*' | paste - - -
grep host_timing $OUT/one_vfirst_timing.log | head -40 | tail -20
