#!/bin/bash
# Run GPU steps given as arguments, each "name:seconds:command ...", in order.
# A step that fails with a test failure (exit 1) does not stop the chain; any
# other non-zero status (fault, abort, timeout, signal) ends it there.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
