# round 5: fused select chain + MC + RCCL split verification; sims at the new defaults
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mc_gpu.py tests/test_loopback_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r5d_tests_a.txt 2>&1
soft timeout -k 10 600 python -u -m pytest tests/test_multigpu_gpu.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r5d_tests_mgpu.txt 2>&1
timeout -k 10 400 python -u bench.py --simulate-world 8 --sim-all --steps 10 --warmup 5 > gpurun_out/r5d_sim8_r50.jsonl 2> gpurun_out/r5d_sim8_r50.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5d_sim8_alex.jsonl 2> gpurun_out/r5d_sim8_alex.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5d_bench.json 2> gpurun_out/r5d_bench.err
