# round 5: fewer ATen launches in the CIFAR graph step (BN gamma/beta into the arena, the image
# conv's padded input kept for backward, post-ReLU pool on the relu-pool kernels, fused-loss
# correctness) — full GPU suite, CIFAR benches, step profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5cn_suite.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5cn_cifar.jsonl 2>> gpurun_out/r5cl.err
done
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5cn_sim8_alex.jsonl 2>> gpurun_out/r5cl.err
bash scripts/prof_cifar_steps.sh anchor alexnet vgg16 > gpurun_out/r5cn_prof_cifar.txt 2>&1
