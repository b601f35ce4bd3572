# A/B variants of the units kernel (build container: `tools/ab_units.sh build`;
# GPU box: `tools/ab_units.sh run [configs...]`).  Each variant is the product
# library with crc32c_kernels.hip rebuilt under extra -D flags; runs are
# interleaved, two passes per variant.  VARIANTS="name:-DX+-DY ..." overrides.
set -e
cd "$(dirname "$0")/.."
V=${VARIANTS:-"base: late:-DLSBM_STORE_LATE nostore:-DLSBM_DIAG_NO_STORE"}
OBJS="build/csrc/crc32c_engine.o build/csrc/crc32c_host.o build/csrc/table_checksum.o build/csrc/log_checksum.o build/csrc/status.o build/csrc/bloom_kernels.o build/csrc/bloom_engine.o build/csrc/bloom_host.o build/csrc/filter_block.o build/csrc/snappy_kernels.o build/csrc/snappy_engine.o build/csrc/block_compression.o build/csrc/host_session.o"
if [ "$1" = build ]; then
  mkdir -p build/abl
  for v in $V; do
    name=${v%%:*}; flags=$(echo ${v#*:} | tr "+" " ")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden $flags \
      -c -o build/abl/k_$name.o ${SRC:-lsbm_amd/csrc/crc32c_kernels.hip} &
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
      LSBM_LIB_PATH=build/abl/lib_$name.so timeout -k 10 200 python -u tools/bench_configs.py ${@:-sst4118 config4}
    done
  done
fi
