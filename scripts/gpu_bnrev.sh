# BN backward apply passes last-to-first (Infinity Cache reuse after the reduce pass): BN / block
# tests, then bench A/B (LWAAAI_BN_REVERSE=1 default vs 0), interleaved.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py tests/test_kernels_gpu.py > gpurun_out/rv_tests.log 2>&1 || { tail -30 gpurun_out/rv_tests.log; exit 1; }
tail -2 gpurun_out/rv_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/rv_$tag.log 2>&1 || { tail gpurun_out/rv_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/rv_$tag.log)"
}
run rev LWAAAI_BN_REVERSE=1
run fwd LWAAAI_BN_REVERSE=0
run rev2 LWAAAI_BN_REVERSE=1
run fwd2 LWAAAI_BN_REVERSE=0
