#!/bin/bash
# Round-end evidence on one GPU, shipped tuning table (no LWAAAI_TUNE_FILE): the headline bench
# twice (the printed top-1 must be identical) and the two-rank RCCL tests on the shared card
# (scripts/bench_matrix.sh is its own call). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
unset LWAAAI_TUNE_FILE
STEPS="bench1:420:python -u bench.py;;bench2:420:python -u bench.py;;\
mgpu:600:LWAAAI_TEST_SHARE_GPU=1 python -u -m pytest tests/test_multigpu_gpu.py -x -v \
--timeout 280 --timeout-method thread" bash scripts/gpu_steps.sh
