# Units-kernel (ragged path) ablations on config 4.
#   build (build container): tools/ablate_units.sh build
#   run (GPU box):           tools/ablate_units.sh run [variants...]
# Each variant is a full library; bench_configs.py config4 loads it through
# LSBM_LIB_PATH.  Diagnostic variants compute wrong CRCs (only time matters).
set -e
cd "$(dirname "$0")/.."
V=${V:-"base: noshift:-DLSBM_ABL_U_NOSHIFT nomerge:-DLSBM_ABL_U_NOMERGE nofix:-DLSBM_ABL_U_NOFIX"}
if [ "$1" = build ]; then
  mkdir -p build/abl_u
  for v in $V; do
    name=${v%%:*}; flags=$(echo ${v#*:} | tr "+" " ")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -munsafe-fp-atomics $flags \
      -c -o build/abl_u/k_$name.o lsbm_amd/csrc/crc32c_kernels.hip
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl_u/lib_$name.so \
      build/abl_u/k_$name.o build/csrc/crc32c_engine.o build/csrc/crc32c_host.o build/csrc/table_checksum.o
  done
else
  shift
  names=${*:-$(for v in $V; do echo -n "${v%%:*} "; done)}
  for pass in 1 2; do
    for name in $names; do
      echo -n "$name pass $pass: "
      LSBM_LIB_PATH=$PWD/build/abl_u/lib_$name.so timeout -k 10 300 python3 tools/bench_configs.py config4 | grep config4
    done
  done
fi
