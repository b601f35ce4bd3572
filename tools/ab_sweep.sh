#!/bin/bash
# A/B of the chunked sweep's chunk size (LSBM_SWEEP_CHUNK_BLOCKS; 0 = one
# range per wave), interleaved, two passes: tools/ab_sweep.sh "64 0 32" configs...
set -e
cd "$(dirname "$0")/.."
V=$1
shift
for pass in 1 2; do
  for v in $V; do
    echo "== chunk $v pass $pass"
    LSBM_SWEEP_CHUNK_BLOCKS=$v timeout -k 10 300 python -u tools/bench_configs.py "$@"
  done
done
