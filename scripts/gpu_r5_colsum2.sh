# round 5: BN forward finalize folding the statistics rows in place, up to how many rows
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 500 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5c2_tests.txt 2>&1
for r in 1 2; do
  for m in 1024 2048 8192; do
    LWAAAI_COLSUM_DIRECT_MAX=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5c2_$m.jsonl 2>> gpurun_out/r5c2.err
  done
done
for m in 1024 2048 8192; do
  LWAAAI_COLSUM_DIRECT_MAX=$m timeout -k 10 300 python -u bench_cifar.py --config anchor --steps 30 --warmup 8 >> gpurun_out/r5c2_cifar_$m.jsonl 2>> gpurun_out/r5c2.err
done
