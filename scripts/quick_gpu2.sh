#!/bin/bash
# One gpurun call after a change to the CIFAR / loss paths: the affected GPU tests, the CIFAR
# benches and the ResNet-50 bench. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/quick2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_xent_gpu.py tests/test_fused_bn_gpu.py tests/test_conv_gpu.py tests/test_gemm_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench_cifar.py --config all --steps 30 --warmup 8 > $O/cifar.log 2>&1 || { tail -20 $O/cifar.log; exit 1; }
grep -o '"metric": "[^"]*", "value": [0-9.]*' $O/cifar.log
timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $O/bench.log
