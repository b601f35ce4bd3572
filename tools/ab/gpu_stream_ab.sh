#!/bin/bash
# A/B of the ragged kernels on the device-resident configs (tools/bench_configs.py):
# LSBM_RAGGED_KERNEL=stream (every eligible batch) against =units, interleaved.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
W=${WHICH:-"wal units4k sst4118 config4"}
for pass in 1 2; do
  LSBM_RAGGED_KERNEL=stream timeout -k 10 400 python -u tools/bench_configs.py $W > gpurun_out/ab/stream_p$pass.log 2>&1 || { echo "stream pass $pass failed"; tail -5 gpurun_out/ab/stream_p$pass.log; exit 1; }
  LSBM_RAGGED_KERNEL=units timeout -k 10 400 python -u tools/bench_configs.py $W > gpurun_out/ab/units_p$pass.log 2>&1 || { echo "units pass $pass failed"; tail -5 gpurun_out/ab/units_p$pass.log; exit 1; }
done
for f in gpurun_out/ab/*.log; do echo "== $f"; cat $f; done
