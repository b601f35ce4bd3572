#!/bin/bash
# FinishFilterBlocks' phases on a 10M-write db_bench database (LSBM_HOST_TIMING=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5_filters; mkdir -p $OUT
g++ -O2 -std=c++17 -pthread -I include tools/db_check_gpu.cc -L lsbm_amd -llsbm_crc32c -Wl,-rpath,$PWD/lsbm_amd -o $OUT/db_check_gpu || exit 1
A="--benchmarks=separate --write_workload=counter --writes=10000000 --value_size=100 --write_key_from=0 --write_key_upto=10000000 --key_from=0 --key_upto=10000000 --read_key_from=0 --read_key_upto=10000000 --writespeed=-1 --readspeed=0 --random_reads=0 --read_threads=0 --countdown=600 --block_cache_size=0 --histogram=0"
mkdir -p /tmp/dbf && timeout -k 10 300 oracle/_ref/db_bench --db=/tmp/dbf $A > /dev/null 2>&1 || exit 1
timeout -k 10 120 oracle/_ref/db_verify /tmp/dbf --filters > $OUT/ref.log 2>&1
for i in 1 2; do
  LSBM_HOST_TIMING=1 timeout -k 10 120 $OUT/db_check_gpu /tmp/dbf 0 --filters > $OUT/gpu_new_$i.log 2>&1 || exit 1
  LD_LIBRARY_PATH=$PWD/build/r5ab/filt_old LSBM_HOST_TIMING=1 timeout -k 10 120 $OUT/db_check_gpu /tmp/dbf 0 --filters > $OUT/gpu_old_$i.log 2>&1 || exit 1
done
grep -o '"filters_ms": [0-9.]*' $OUT/ref.log
for f in $OUT/gpu_*.log; do echo "$f $(grep -o '"filters_identical": [0-9]*\|"false_negatives": [0-9]*\|"filters_feed_ms": [0-9.]*\|"filters_finish_ms": [0-9.]*' $f | tr '\n' ' ')"; grep -o '"host_timing": "FinishFilterBlocks"[^}]*' $f; done; true
