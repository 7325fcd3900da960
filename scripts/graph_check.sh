#!/bin/bash
# HIP-graph step: capture probe, GPU tests, bench with graph on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probes/graph_capture_probe.py > gpurun_out/probe.log 2>&1
echo probe_rc=$?; grep -v "^\s*$" gpurun_out/probe.log | tail -12
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_graph_step_gpu.py > gpurun_out/graph_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -12 gpurun_out/graph_test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in on off; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --graph $mode > gpurun_out/bench_$mode.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' gpurun_out/bench_$mode.log | tr '\n' ' '; echo
done
