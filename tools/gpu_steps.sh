#!/bin/bash
# The one GPU-session runner: each argument is a step "name:seconds:command
# ...", run in order under its own time limit, output in
# gpurun_out/$RUN/<name>.log and a one-line summary per step (with the bench
# line's value, if any) in gpurun_out/$RUN/steps.log.  A step that fails with
# a test failure (exit 1) does not stop the chain; any other non-zero status
# (fault, abort, timeout, signal) ends it there.
#   RUN=r6s3 bash tools/gpu_steps.sh "pytest:600:python -u -m pytest tests -m gpu -x -q" \
#       "bench:300:python bench.py" "bs:300:BSSL_AMD_GCM_MODE=bs python bench.py"
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-steps}
mkdir -p "$O"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  echo "[$(date +%T)] start $name" | tee -a "$O/steps.log"
  timeout -k 10 "$t" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' "$O/$name.log" | head -1)" | tee -a "$O/steps.log"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
