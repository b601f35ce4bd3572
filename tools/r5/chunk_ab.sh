#!/bin/bash
# Staging chunk A/B: 64 MiB (in tree) vs 16 MiB (build/r5ab/chunk16) on the
# whole-database check (first and repeated VerifyTables) and the host layers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5_chunk; mkdir -p $OUT
g++ -O2 -std=c++17 -pthread -I include tools/db_check_gpu.cc -L lsbm_amd -llsbm_crc32c -Wl,-rpath,$PWD/lsbm_amd -o $OUT/db_check_gpu || exit 1
A="--benchmarks=separate --write_workload=counter --writes=10000000 --value_size=100 --write_key_from=0 --write_key_upto=10000000 --key_from=0 --key_upto=10000000 --read_key_from=0 --read_key_upto=10000000 --writespeed=-1 --readspeed=0 --random_reads=0 --read_threads=0 --countdown=600 --block_cache_size=0 --histogram=0"
mkdir -p /tmp/dbchunk && timeout -k 10 300 oracle/_ref/db_bench --db=/tmp/dbchunk $A > /dev/null 2>&1 || exit 1
for p in 1 2; do
  for v in c64 c16; do
    lp=""; [ $v = c16 ] && lp=$PWD/build/r5ab/chunk16
    echo "== $v pass $p" >> $OUT/ab.log
    LD_LIBRARY_PATH=$lp timeout -k 10 120 $OUT/db_check_gpu /tmp/dbchunk 0 >> $OUT/ab.log 2>&1 || exit 1
    LD_LIBRARY_PATH=$lp timeout -k 10 300 build/bench_host_layers 200 1024 >> $OUT/ab.log 2>&1 || exit 1
  done
done
echo done
