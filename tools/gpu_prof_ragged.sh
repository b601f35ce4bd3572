#!/bin/bash
# PMC passes (tools/gpu_units_pmc.sh) over tools/prof_ragged.py workloads, for
# the stream kernel and (LSBM_RAGGED_KERNEL=units) the units kernel.
export TMPDIR=/tmp
for w in ${WHICH:-wal units4k}; do
  LSBM_RAGGED_KERNEL=stream ./tools/gpu_units_pmc.sh gpurun_out/prof/$w python3 tools/prof_ragged.py $w || exit 1
  [ -n "$NO_UNITS" ] || LSBM_RAGGED_KERNEL=units ./tools/gpu_units_pmc.sh gpurun_out/prof/${w}_units python3 tools/prof_ragged.py $w || exit 1
done
for d in gpurun_out/prof/*; do echo "== $d"; python3 tools/pmc_summary.py $d; done
