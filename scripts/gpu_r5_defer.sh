# round 5: deferred split-K reduces (one launch per flush) — tests, ResNet-50 A/B, step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 600 python -u -m pytest tests/test_block_gpu.py tests/test_graph_step_gpu.py tests/test_topk_parity_gpu.py tests/test_fused_sgd_gpu.py tests/test_engine_invariants_gpu.py tests/test_loopback_gpu.py tests/test_fp16_gpu.py tests/test_gemm_gpu.py tests/test_conv_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5d_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5d_on.jsonl 2>> gpurun_out/r5d.err
  LWAAAI_SPLITK_DEFER=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5d_off.jsonl 2>> gpurun_out/r5d.err
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 > gpurun_out/r5d_bench_acc.json 2>> gpurun_out/r5d.err
bash scripts/prof_step.sh r5d > gpurun_out/r5d_prof_step.txt 2>&1
