# round 5: lazy [K][C] dgrad weight pack — tests, bench, step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py tests/test_fp16_gpu.py tests/test_mf32_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5l2_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5l2_bench.jsonl 2>> gpurun_out/r5l2.err
done
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5l2_cifar.jsonl 2>> gpurun_out/r5l2.err
bash scripts/prof_step.sh r5l2 > gpurun_out/r5l2_prof_step.txt 2>&1
