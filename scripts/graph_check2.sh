#!/bin/bash
# Graph-mode GPU tests (ImageNet + CIFAR trainers), CIFAR benches graph on/off, ResNet-50 bench,
# then the 24-epoch ResNet-9 CLI runs (demo.ipynb protocol on synthetic data).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_graph_step_gpu.py > gpurun_out/graph_test.log 2>&1
rc=$?; echo test_rc=$rc; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/graph_test.log | tail -14
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in on off; do
  timeout -k 10 300 python bench_cifar.py --graph $mode > gpurun_out/cifar_$mode.log 2>&1 || exit $?
  grep -o '"metric": "[^"]*"\|"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' gpurun_out/cifar_$mode.log | tr '\n' ' '; echo
done
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_on.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hip_graph": [a-z]*' gpurun_out/bench_on.log | tr '\n' ' '; echo
timeout -k 10 400 python CIFAR10/dawn.py --synthetic -w 1 --epochs 24 --log_dir gpurun_out/dawn24_none > gpurun_out/dawn24_none.log 2>&1 || exit $?
tail -4 gpurun_out/dawn24_none.log
timeout -k 10 400 python CIFAR10/dawn.py --synthetic -w 1 --epochs 24 -c layerwise --method Topk -K 0.01 --log_dir gpurun_out/dawn24_topk > gpurun_out/dawn24_topk.log 2>&1 || exit $?
tail -4 gpurun_out/dawn24_topk.log
