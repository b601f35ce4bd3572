#!/bin/bash
# Round 4: host layers and one table, new worker pool (atomic piece claims)
# against round 4's earlier pool (build/abl/oldpool), interleaved, two passes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4_check13}
mkdir -p $OUT
for p in 1 2; do
  for v in new oldpool; do
    if [ $v = new ]; then L=""; else L="$PWD/build/abl/$v"; fi
    LD_LIBRARY_PATH=$L timeout -k 10 300 build/bench_host_layers 1000 1024 > $OUT/host_${v}_p$p.log 2>&1 || exit 1
    LD_LIBRARY_PATH=$L timeout -k 10 180 build/bench_one_table 100 4 > $OUT/one_${v}_p$p.log 2>&1 || exit 1
  done
done
for f in $OUT/host_*.log; do echo "== $f"; grep -o '"pinned": [01], "seal": "OK", "seal_s": [0-9.]*, "seal_GBps": [0-9.]*, "verify": "OK", "verify_s": [0-9.]*, "verify_GBps": [0-9.]*' $f; grep -o '"what": "wal".*"verify_GBps": [0-9.]*' $f | cut -c1-200; done
for f in $OUT/one_*.log; do echo "== $f"; grep -E '"(seal|verify)_(pageable|locked)"|host_copy' $f | grep -o '"what": "[a-z_0-9A-Z]*"\|"p50_ms": [0-9.]*' | paste - - ; done
