#!/bin/bash
# Same-box A/B of device entry points by HIP events (tools/roofline_all.py's
# events_ms, which agrees with rocprof's kernel average within ~1%): for each
# pass, each entry and each variant, one process.
#
#   tools/ab/events_ab.sh OUT "ENTRIES" "VARIANTS" [PASSES=2]
#
# VARIANTS as in tools/ab/interleave.sh: `name`, `name=lib:PATH`, `name=env:K=V[,K=V]`.
# Example (round 6, profiles/r06/events_ab/): the round-5 library against this one
#   tools/ab/events_ab.sh gpurun_out/r6ab "fixed4k sst_verify config4" "r06 r05=lib:build/r6/r05/liblsbm_crc32c.so"
set -o pipefail
OUT=$1; ENTRIES=$2; VARIANTS=$3; PASSES=${4:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p "$OUT"
for p in $(seq 1 "$PASSES"); do
  for e in $ENTRIES; do
    for v in $VARIANTS; do
      n=${v%%=*}; s=""; case "$v" in *=*) s=${v#*=} ;; esac
      case "$s" in
        lib:*) pre="env LSBM_LIB_PATH=${s#lib:}" ;;
        env:*) pre="env $(echo "${s#env:}" | tr ',' ' ')" ;;
        *) pre="" ;;
      esac
      line=$($pre timeout -k 10 300 python3 tools/roofline_all.py "$e" 2>>"$OUT/stderr.log" | tail -1)
      rc=$?; [ $rc -eq 0 ] || { echo "$e $n pass $p rc=$rc"; exit $rc; }
      echo "$p $e $n $line" | tee -a "$OUT/ab.log"
    done
  done
done
python3 - "$OUT/ab.log" <<'EOF'
import json, sys, collections
r = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    p, e, n, js = ln.split(" ", 3)
    r[(e, n)].append(json.loads(js)["events_pct_hbm"])
for (e, n), v in sorted(r.items()):
    print(f"{e:12s} {n:10s} " + " / ".join(f"{x:.2f}" for x in v))
EOF
