# Build ablation variants of the library (build container): tools/ablate.sh build
# Run them (GPU box):                                        tools/ablate.sh run
set -e
cd "$(dirname "$0")/.."
V="base:-DLSBM_PF=4 static:-DLSBM_ABL_STATIC pf3:-DLSBM_PF=3 diag:-DLSBM_DIAG_STAMPS"
if [ "$1" = build ]; then
  mkdir -p build/abl
  for v in $V; do
    name=${v%%:*}; flags=$(echo ${v#*:} | tr "+" " ")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden $flags \
      -c -o build/abl/k_$name.o lsbm_amd/csrc/crc32c_kernels.hip
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl/lib_$name.so \
      build/abl/k_$name.o build/csrc/crc32c_engine.o build/csrc/crc32c_host.o
  done
  /opt/rocm/bin/hipcc -O2 -std=c++17 -o build/abl/driver tools/ablate_driver.cc -ldl
elif [ "$1" = sweep ]; then
  for v in ${2:-base pf2}; do ABL_SWEEP=1 ABL_NMAX=8388608 timeout -k 10 300 build/abl/driver build/abl/lib_$v.so; done
else
  args=""
  for v in $V; do args="$args build/abl/lib_${v%%:*}.so"; done
  timeout -k 10 300 build/abl/driver $args
fi
