#!/bin/bash
# Level 1 vs the GPU ends (tests/cpp/ref_compaction_gpu.cc, _l1 build): pooled
# page-locked images, pooled but not page-locked (LSBM_TABLE_REGISTER=0), and
# unpooled (LSBM_POOL_IMAGES=0); three interleaved passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5_compaction2; mkdir -p $OUT
for p in 1 2 3; do
  for v in pooled pooled_unlocked unpooled; do
    case $v in pooled) e="";; pooled_unlocked) e="LSBM_TABLE_REGISTER=0";; unpooled) e="LSBM_POOL_IMAGES=0";; esac
    echo "== $v pass $p" >> $OUT/compaction.log
    env $e timeout -k 10 300 oracle/_ref/gpu_compaction_l1 4 16 16 >> $OUT/compaction.log 2>&1 || { echo "$v failed"; exit 1; }
  done
done
grep -E "^==|^OK|^FAIL" $OUT/compaction.log
