#!/bin/bash
# gpurun with retries on infrastructure-side transients only (no box / slot / box not prepared); never on a run's own failure.
out=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out; then sleep 90; continue; fi
  exit $rc
done
exit $rc
