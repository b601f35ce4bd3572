#!/bin/bash
# Event counters of the stream kernel (crc32c_stream.hip built with
# -DLSBM_STREAM_STATS): wave-rows, slow wave-rows, general half-steps, ...
#   build (build container): tools/stream_stats.sh build
#   run (GPU box):           tools/stream_stats.sh run [workloads...]
set -e
cd "$(dirname "$0")/.."
if [ "$1" = build ]; then
  make -C lsbm_amd/csrc -j8 >/dev/null
  mkdir -p build/abl_s
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -munsafe-fp-atomics \
    -DLSBM_STREAM_STATS -c -o build/abl_s/stream_stats.o lsbm_amd/csrc/crc32c_stream.hip
  objs=$(ls build/csrc/*.o | grep -v crc32c_stream.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl_s/lib_stats.so build/abl_s/stream_stats.o $objs
else
  shift
  for w in ${*:-wal walseal units4k sst c4}; do
    LSBM_RAGGED_KERNEL=stream LSBM_LIB_PATH=$PWD/build/abl_s/lib_stats.so timeout -k 10 200 python3 tools/prof_ragged.py $w --reps 1 --stats
  done
fi
