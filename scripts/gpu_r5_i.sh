# round 5: headline bench (calibrated accuracy run), MC config row, world-8 simulations of
# BASELINE configs 3-5, step profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5i_tests.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r5i_bench_topk_noacc.json 2>> gpurun_out/r5i_bench.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 --ef --ef-dense-below 4096 --momentum-correction > gpurun_out/r5i_bench_mc.json 2>> gpurun_out/r5i_bench.err
timeout -k 10 400 python -u bench.py --simulate-world 8 --sim-all --steps 10 --warmup 5 > gpurun_out/r5i_sim8_r50.jsonl 2> gpurun_out/r5i_sim8.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5i_sim8_alex.jsonl 2>> gpurun_out/r5i_sim8.err
timeout -k 10 300 python -u bench_cifar.py --config vgg16 --steps 30 --warmup 8 > gpurun_out/r5i_bench_vgg.jsonl 2> gpurun_out/r5i_bench_vgg.err
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5i_prof_cifar.txt 2>&1
bash scripts/prof_step.sh r5i > gpurun_out/r5i_prof_step.txt 2>&1
