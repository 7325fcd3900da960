#!/bin/bash
# Generic one-call GPU runner: STEPS="name:timeout:cmd;;name:timeout:cmd" — each step under its
# own time limit, output to gpurun_out/<name>.log, stop at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/summary.log
IFS=$'\n'
for spec in $(echo "$STEPS" | sed 's/;;/\n/g'); do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($to s): $cmd" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -6 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
done
echo done
