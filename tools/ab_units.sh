#!/bin/bash
# A/B variants of one kernel file (build container: `tools/ab_units.sh build`;
# GPU box: `tools/ab_units.sh run [configs...]`).  Each variant is the product
# library with that kernel file rebuilt under extra -D flags (or from another
# source, SRC=...); runs are interleaved, two passes per variant.
#   VARIANTS="name:-DX+-DY ..."   the variants
#   KFILE=crc32c_kernels|bloom_kernels|snappy_kernels   (default crc32c_kernels)
#   BENCH="python -u tools/bench_configs.py"            the command run per variant
set -e
cd "$(dirname "$0")/.."
V=${VARIANTS:-"base:"}
K=${KFILE:-crc32c_kernels}
ALL="crc32c_kernels crc32c_engine crc32c_host table_checksum log_checksum status bloom_kernels bloom_engine bloom_host filter_block snappy_kernels snappy_engine block_compression host_session"
OBJS=""
for o in $ALL; do [ "$o" = "$K" ] || OBJS="$OBJS build/csrc/$o.o"; done
if [ "$1" = build ]; then
  mkdir -p build/abl
  for v in $V; do
    name=${v%%:*}; flags=$(echo ${v#*:} | tr "+" " ")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -munsafe-fp-atomics $flags \
      -c -o build/abl/k_$name.o ${SRC:-lsbm_amd/csrc/$K.hip} &
  done
  wait
  for v in $V; do
    name=${v%%:*}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/lib_$name.so build/abl/k_$name.o $OBJS
  done
else
  shift
  for pass in 1 2; do
    for v in $V; do
      name=${v%%:*}
      echo "== $name pass $pass"
      if [ -n "$BENCH" ]; then
        LSBM_LIB_PATH=build/abl/lib_$name.so timeout -k 10 200 $BENCH "$@"
      else
        LSBM_LIB_PATH=build/abl/lib_$name.so timeout -k 10 200 python -u tools/bench_configs.py ${@:-sst4118 config4}
      fi
    done
  done
fi
