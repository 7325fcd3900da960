# round 5: batched-load select chain (k_hist / k_count_sel fast path, float4 residual stores,
# unsplit pass 0): tests, benches, world-8 sims, MC A/B, step profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_mc_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py tests/test_topk_parity_gpu.py tests/test_ef_gpu.py tests/test_overflow_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5y_tests.txt 2>&1
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5y_bench_cifar.jsonl 2> gpurun_out/r5y_bench_cifar.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5y_sim8_alex.jsonl 2> gpurun_out/r5y_sim8.err
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --steps 20 --warmup 5 > gpurun_out/r5y_sim8_r50.jsonl 2>> gpurun_out/r5y_sim8.err
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5y_ab_mc.jsonl 2>> gpurun_out/r5y_ab.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 --ef --ef-dense-below 4096 --momentum-correction >> gpurun_out/r5y_ab_mc.jsonl 2>> gpurun_out/r5y_ab.err
done
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5y_prof_cifar.txt 2>&1
