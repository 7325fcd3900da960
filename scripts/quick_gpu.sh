#!/bin/bash
# One gpurun call for a change to the GEMM core / its users: GEMM, conv and linear tests, the
# tile sweep, the Linear-vs-BLAS microbench and a 1-GPU bench. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_block_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python scripts/tile_sweep.py > $O/tile_sweep.log 2>&1 || exit 1
timeout -k 10 300 python scripts/linear_vs_blas.py > $O/linear_vs_blas.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $O/bench.log
