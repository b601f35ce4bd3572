#!/bin/bash
export TMPDIR=/tmp
VARIANTS="pre2 v3" WHICH="wal units4k config4" bash tools/gpu_lean_ab.sh || exit $?
NO_UNITS=1 WHICH=wal bash tools/gpu_prof_ragged.sh > gpurun_out/prof_wal.log 2>&1; echo "prof rc=$?"
