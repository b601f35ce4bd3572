#!/bin/bash
# A/B library: build/abl/NAME/liblsbm_crc32c.so = the product objects
# (build/csrc, from `make -C lsbm_amd/csrc`) with one kernel source recompiled
# under extra defines.  Load it through LSBM_LIB_PATH.
#   tools/ab/variant.sh NAME bloom_kernels "-DLSBM_PROBE_HANDLE_AHEAD=0"
set -e
NAME=$1; SRC=$2; DEFS=$3
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
D=${ABL_DIR:-$ROOT/build/abl}/$NAME; mkdir -p $D
make -s -C $ROOT/lsbm_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -fvisibility=hidden -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -munsafe-fp-atomics -DLSBM_DIAG_BUILD $DEFS -c -o $D/$SRC.o $ROOT/lsbm_amd/csrc/$SRC.hip
OBJS=$(ls $ROOT/build/csrc/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/liblsbm_crc32c.so $OBJS $D/$SRC.o
echo "$D/liblsbm_crc32c.so"
