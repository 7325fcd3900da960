# Mixed-layout big tiles: GEMM tests, Linear vs BLAS, ResNet-50 bench, CIFAR configs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py > gpurun_out/mx_tests.log 2>&1 || { tail -30 gpurun_out/mx_tests.log; exit 1; }
tail -2 gpurun_out/mx_tests.log
timeout -k 10 300 python scripts/linear_vs_blas.py > gpurun_out/linear_vs_blas_mixed.log 2>&1 || { tail -5 gpurun_out/linear_vs_blas_mixed.log; exit 1; }
grep -E "vgg16.fc1|alexnet.fc2|layer" gpurun_out/linear_vs_blas_mixed.log
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/mx_bench.log 2>&1 || { tail gpurun_out/mx_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/mx_bench.log
timeout -k 10 600 python bench_cifar.py --config all > gpurun_out/mx_cifar.log 2>&1 || { tail -20 gpurun_out/mx_cifar.log; exit 1; }
grep -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/mx_cifar.log
