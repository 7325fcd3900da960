# round 5: BN forward finalize folding one-row-per-block statistics rows in place (no k_colsum)
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 500 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py tests/test_topk_parity_gpu.py tests/test_gemm_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5c_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5c_on.jsonl 2>> gpurun_out/r5c.err
  LWAAAI_COLSUM_DIRECT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5c_off.jsonl 2>> gpurun_out/r5c.err
done
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5c_cifar_on.jsonl 2>> gpurun_out/r5c.err
LWAAAI_COLSUM_DIRECT=0 timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5c_cifar_off.jsonl 2>> gpurun_out/r5c.err
