#!/bin/bash
# One compaction three ways (tests/cpp/ref_compaction_gpu.cc): the reference,
# Level 1 and the GPU ends, the GPU ends with pooled page-locked images
# (default) and without (LSBM_POOL_IMAGES=0); two interleaved passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5_compaction; mkdir -p $OUT
for p in 1 2; do
  for v in pooled unpooled; do
    for b in gpu_compaction gpu_compaction_l1; do
      e=""; [ $v = unpooled ] && e="LSBM_POOL_IMAGES=0"
      echo "== $b $v pass $p" >> $OUT/compaction.log
      env $e timeout -k 10 300 oracle/_ref/$b 4 16 16 >> $OUT/compaction.log 2>&1 || { echo "$b $v failed"; exit 1; }
    done
  done
done
grep -E "^==|^OK|^FAIL" $OUT/compaction.log
