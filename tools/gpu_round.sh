# One GPU call, several independent steps: each runs under its own time limit;
# a step that fails its checks (rc 1) does not stop the next, anything else
# (timeout, abort, fault) ends the call.
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  echo "=== $step"
  bash "$step"
  rc=$?
  echo "=== $step rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
