# round 5: split threshold + equal-digit histogram; sims, benches, profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_mc_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5r_tests.txt 2>&1
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --steps 20 --warmup 5 > gpurun_out/r5r_sim8_r50.jsonl 2> gpurun_out/r5r_sim8.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5r_sim8_alex.jsonl 2>> gpurun_out/r5r_sim8.err
timeout -k 10 400 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5r_bench_cifar.jsonl 2> gpurun_out/r5r_bench_cifar.err
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5r_bench.json 2> gpurun_out/r5r_bench.err
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5r_prof_cifar.txt 2>&1
bash scripts/prof_step.sh r5r > gpurun_out/r5r_prof_step.txt 2>&1
