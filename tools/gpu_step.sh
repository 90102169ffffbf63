#!/bin/bash
# Run GPU steps in order; stop at the first step that timed out, aborted,
# crashed or was killed (exit 124/134/137/139 or >128), continue past an
# ordinary failure (a failed test).  Each step: a shell string run under its
# own timeout.  usage: tools/gpu_step.sh SECONDS 'cmd1' SECONDS 'cmd2' ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
worst=0
while [ $# -ge 2 ]; do
  t=$1; c=$2; shift 2
  echo "== step: $c" >&2
  timeout -k 10 $t bash -c "$c"
  rc=$?
  echo "== rc=$rc" >&2
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "stopping after rc=$rc" >&2; exit $rc; fi
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
