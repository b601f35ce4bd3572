#!/bin/bash
# Rehearsal on the last library (WAL epilogue without length re-reads).
export TMPDIR=/tmp
bash tools/gpu_final.sh || exit $?
OUT=gpurun_out/final4; mkdir -p $OUT
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.log $OUT/
