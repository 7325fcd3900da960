#!/bin/bash
# One gpurun call: GPU tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first step that faults / aborts / times out (exit >= 124 or signal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/summary.log
run build 600 python -m layer_wise_aaai20_amd.csrc.build
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps $STEPS --warmup 8
if [ "${PROFILE:-1}" = "1" ]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 5 --warmup 3
fi
echo done
