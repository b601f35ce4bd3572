#!/bin/bash
export TMPDIR=/tmp
VARIANTS="v3" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh || exit $?
bash tools/gpu_r3_host2.sh
