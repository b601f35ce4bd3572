#!/bin/bash
# PMC of the final seal paths: the SSTable seal (units kernel, dense CRCs +
# per-wave trailer merges) and the WAL seal with d_masked (stream kernel,
# deferred headers), against the verifies on the same images.
export TMPDIR=/tmp
rm -rf gpurun_out/prof
WHICH="sstseal sst walseal wal" NO_UNITS=1 bash tools/gpu_prof_ragged.sh > gpurun_out/sealpmc.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v "^pass" gpurun_out/sealpmc.log | tail -60
exit $rc
