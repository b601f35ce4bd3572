#!/bin/bash
# Round-3 rehearsal, part B: the ragged / SSTable / WAL configs, the bloom
# lines with PMC traffic, the host layers.
export TMPDIR=/tmp
OUT=gpurun_out/finalB
mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_configs.py config1 config3 config4 sst4118 wal host > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; python3 tools/ab_summary.py $OUT/configs.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/bloom_traffic bash tools/gpu_bloom_traffic.sh > $OUT/bloom_traffic.log 2>&1
rc=$?; echo "bloom traffic rc=$rc"; tail -3 $OUT/bloom_traffic.log; [ $rc -eq 0 ] || exit $rc
cp profiles/bloom_traffic.json $OUT/
timeout -k 10 300 python -u tools/bench_bloom.py > $OUT/bench_bloom.log 2>&1
rc=$?; echo "bloom rc=$rc"; cut -c1-300 $OUT/bench_bloom.log; [ $rc -eq 0 ] || exit $rc
LSBM_HOST_TIMING=1 timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_layers.log 2> $OUT/host_timing.log
rc=$?; echo "host layers rc=$rc"; cut -c1-300 $OUT/host_layers.log; [ $rc -eq 0 ] || exit $rc
bash tools/stream_stats.sh run wal walseal sst > $OUT/stream_stats.log 2>&1
rc=$?; echo "stream stats rc=$rc"; grep -v "^W\|amdgpu.ids" $OUT/stream_stats.log; exit $rc
