# One-launch colsum + finalize v2: tests with it on, bench A/B, then the GEMM / Linear benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LWAAAI_COLSUM_FUSED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py tests/test_conv_gpu.py > gpurun_out/cs2_tests.log 2>&1 || { tail -30 gpurun_out/cs2_tests.log; exit 1; }
tail -2 gpurun_out/cs2_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/cs2_$tag.log 2>&1 || { tail gpurun_out/cs2_$tag.log; exit 1; }
  echo "$tag ($*): $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/cs2_$tag.log)"
}
run off LWAAAI_COLSUM_FUSED=0
run on LWAAAI_COLSUM_FUSED=1
run off2 LWAAAI_COLSUM_FUSED=0
run on2 LWAAAI_COLSUM_FUSED=1
timeout -k 10 400 python scripts/gemm_big_bench.py > gpurun_out/gemm_big_bench_r3s2.jsonl 2>&1 || { tail -5 gpurun_out/gemm_big_bench_r3s2.jsonl; exit 1; }
timeout -k 10 300 python scripts/linear_vs_blas.py > gpurun_out/linear_vs_blas_r3s2.log 2>&1 || { tail -5 gpurun_out/linear_vs_blas_r3s2.log; exit 1; }
cat gpurun_out/linear_vs_blas_r3s2.log
