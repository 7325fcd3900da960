# round 5: new kernels' tests, CIFAR benches, convergence calibration at the final settings
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 400 python -u -m pytest tests/test_fused_sgd_gpu.py tests/test_kernels_gpu.py tests/test_graph_step_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5o_tests.txt 2>&1
timeout -k 10 400 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5o_bench_cifar.jsonl 2> gpurun_out/r5o_bench_cifar.err
timeout -k 10 600 python -u scripts/convergence_calibrate.py --seeds 0,1,2 > gpurun_out/r5o_convergence_calibration.jsonl 2> gpurun_out/r5o_conv.err
