# round 5: fused decode+SGD, RCCL init rework, multi-rank suite, benches
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 600 python -u -m pytest tests/test_fused_sgd_gpu.py tests/test_mc_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r5e_tests_a.txt 2>&1
soft timeout -k 10 700 python -u -m pytest tests/test_multigpu_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r5e_tests_mgpu.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5e_bench.json 2> gpurun_out/r5e_bench.err
for c in vgg16 alexnet resnet9; do
  timeout -k 10 300 python -u bench_cifar.py --config $c --steps 30 --warmup 8 >> gpurun_out/r5e_bench_cifar.jsonl 2>> gpurun_out/r5e_bench_cifar.err
done
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5e_sim8_alex.jsonl 2> gpurun_out/r5e_sim8_alex.err
