#!/bin/bash
# rocprofv3 kernel trace of a short bench run; the raw trace stays in /tmp (too large to ship
# back), the steady-state per-step breakdown goes to gpurun_out/$TAG_steps.txt.
# usage: scripts/prof_step.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-step}; shift
mkdir -p gpurun_out /tmp/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof/$TAG -o run --output-format csv \
  -- python bench.py --steps 6 --warmup 6 --acc-steps 0 "$@" > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
KT=$(find /tmp/prof/$TAG -name '*kernel_trace.csv' | head -1)
ST=$(find /tmp/prof/$TAG -name '*kernel_stats.csv' | head -1)
cp "$ST" gpurun_out/${TAG}_kernel_stats.csv
SEQ=gpurun_out/${TAG}_seq.txt python scripts/trace_steps.py "$KT" 5 -v > gpurun_out/${TAG}_steps.txt
cat gpurun_out/${TAG}_steps.txt
