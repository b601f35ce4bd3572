#!/bin/bash
# One parameterised A/B runner (replaces round 4's 30 one-off check scripts):
# for each variant, an optional GPU test step, then PASSES interleaved passes
# of a bench command over all variants, each run under its own time limit;
# the first failing step ends the script (no retries: DESIGN/CLAUDE GPU rules).
#
#   tools/ab/interleave.sh OUT "VARIANTS" "TESTS" "BENCH" [PASSES=2]
#
#   OUT       output directory (under gpurun_out/)
#   VARIANTS  space-separated: `name` (the in-tree library, as is),
#             `name=lib:PATH` (LSBM_LIB_PATH=PATH), `name=env:K=V[,K=V]`
#   TESTS     pytest arguments run once per variant ("" = none), e.g.
#             "tests/test_log.py -m gpu"
#   BENCH     the command timed per pass and variant, e.g.
#             "python -u tools/bench_configs.py wal" or "build/bench_one_table 100 4"
#
# Examples (round 5):
#   WAL merge A/B (profiles/r05/wal_ab/):
#     tools/ab/interleave.sh gpurun_out/r5ab "default mpar=lib:build/r5ab/mpar.so lds16=lib:build/r5ab/lds16.so" \
#       "tests/test_log.py tests/test_stream.py -m gpu" "python -u tools/bench_configs.py wal"
#   per-call page locks on / off (profiles/r05/host_cpu/):
#     tools/ab/interleave.sh gpurun_out/r5lock "auto staged=env:LSBM_AUTO_LOCK=0" "" "build/bench_one_table 100 4"
set -o pipefail
OUT=$1; VARIANTS=$2; TESTS=$3; BENCH=$4; PASSES=${5:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p "$OUT"
# run_as NAME SPEC CMD...: CMD with the variant's library / environment
run_as() {
  local spec=$2; shift 2
  case "$spec" in
    lib:*) env LSBM_LIB_PATH="${spec#lib:}" "$@" ;;
    env:*) env $(echo "${spec#env:}" | tr ',' ' ') "$@" ;;
    *) "$@" ;;
  esac
}
spec_of() { case "$1" in *=*) echo "${1#*=}" ;; *) echo "" ;; esac; }
name_of() { echo "${1%%=*}"; }
if [ -n "$TESTS" ]; then
  for v in $VARIANTS; do
    n=$(name_of "$v"); s=$(spec_of "$v")
    run_as "$n" "$s" timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest_$n.log" 2>&1
    rc=$?; echo "$n tests rc=$rc $(tail -1 "$OUT/pytest_$n.log")"; [ $rc -eq 0 ] || exit $rc
  done
fi
for p in $(seq 1 "$PASSES"); do
  for v in $VARIANTS; do
    n=$(name_of "$v"); s=$(spec_of "$v")
    echo "== $n pass $p" >> "$OUT/bench.log"
    run_as "$n" "$s" timeout -k 10 600 $BENCH >> "$OUT/bench.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$n pass $p rc=$rc"; exit $rc; }
  done
done
echo "done: $OUT/bench.log"
