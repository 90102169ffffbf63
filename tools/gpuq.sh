#!/bin/bash
# (tools/gpuq.sh OUT gpurun-args...: the wrapper the builder uses from the container; never on the GPU box)
# retry a gpurun call only while the pool has no free box (rc 3 / transient); never on a command failure
out=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy" $out && [ $rc -ne 0 ]; then sleep 90; continue; fi
  echo "RC=$rc" >> $out
  exit $rc
done
echo "RC=gaveup" >> $out
