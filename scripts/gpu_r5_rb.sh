# round 5: relu_bias_bwd grid by width — tests, CIFAR benches, VGG-16 step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_step_gpu.py tests/test_fused_bn_gpu.py tests/test_conv_gpu.py tests/test_fused_sgd_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5rb_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5rb_cifar.jsonl 2>> gpurun_out/r5rb.err
done
bash scripts/prof_cifar_steps.sh vgg16 > gpurun_out/r5rb_prof_cifar.txt 2>&1
