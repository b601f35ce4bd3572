cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out/r5_dbg
A="--benchmarks=separate --write_workload=counter --writes=1000000 --value_size=100 --write_key_from=0 --write_key_upto=1000000 --key_from=0 --key_upto=1000000 --read_key_from=0 --read_key_upto=1000000 --writespeed=-1 --readspeed=0 --random_reads=0 --read_threads=0 --countdown=600 --block_cache_size=0 --histogram=0"
for i in 1 2 3; do
 for b in db_bench_l1 db_bench_gpu; do
  rm -rf /tmp/d_$b; mkdir /tmp/d_$b
  LSBM_TABLE_STATS=1 timeout -k 5 120 ./oracle/_ref/$b --db=/tmp/d_$b $A > /tmp/o.txt 2> /tmp/e.txt || exit 1
  echo "$b $(grep separate /tmp/o.txt) $(grep lsbm_table_stats /tmp/e.txt)" >> gpurun_out/r5_dbg/log.txt
 done
done
LSBM_TABLE_STATS=1 LSBM_WAIT=spin timeout -k 5 120 ./oracle/_ref/db_bench_gpu --db=/tmp/d_x $A > /tmp/o.txt 2>/tmp/e.txt; echo "spin $(grep separate /tmp/o.txt) $(grep lsbm_table_stats /tmp/e.txt)" >> gpurun_out/r5_dbg/log.txt
cat gpurun_out/r5_dbg/log.txt
