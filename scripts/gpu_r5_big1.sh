# round 5: big-workgroup pass 0 — probe A/B, GPU select tests, and bench A/B (LWAAAI_HIST0_BIG)
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in v0 small0; do
  for n in 2260892 9042734; do
    timeout -k 10 60 build/probe/sp_$v $n 0.01 50 >> gpurun_out/r5b1_probe.txt
  done
  timeout -k 10 60 build/probe/sp_$v 8500000 0.001 50 1 >> gpurun_out/r5b1_probe.txt
done
soft timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_mc_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py tests/test_topk_parity_gpu.py tests/test_ef_gpu.py tests/test_graph_step_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5b1_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5b1_cifar_big.jsonl 2>> gpurun_out/r5b1.err
  LWAAAI_HIST0_BIG=0 timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5b1_cifar_small.jsonl 2>> gpurun_out/r5b1.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5b1_r50_big.jsonl 2>> gpurun_out/r5b1.err
  LWAAAI_HIST0_BIG=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5b1_r50_small.jsonl 2>> gpurun_out/r5b1.err
done
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5b1_sim8_alex.jsonl 2>> gpurun_out/r5b1.err
