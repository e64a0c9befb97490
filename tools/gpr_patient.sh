#!/bin/bash
# gpurun, retried only while the pool reports an infrastructure transient
# (no box / slot / box creation failed: nothing ran, nothing charged); never
# on a run's own failure.  Usage: tools/gpr_patient.sh <log> <gpurun args...>
out=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out; then sleep 120; continue; fi
  exit $rc
done
exit $rc
