# Split-K slices per XCD (tile_split_of): GEMM / conv tests, then bench A/B against a build with
# -DLW_SPLIT_XCD=0 (_lwaaai_C_nox.so), interleaved, plus the op roofline of the new mapping.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_block_gpu.py > gpurun_out/sx_tests.log 2>&1 || { tail -30 gpurun_out/sx_tests.log; exit 1; }
tail -2 gpurun_out/sx_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/sx_$tag.log 2>&1 || { tail gpurun_out/sx_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/sx_$tag.log)"
}
run xcd LWAAAI_X=0
run nox LWAAAI_SO=$GRAFT_REPO_ROOT/layer_wise_aaai20_amd/_lwaaai_C_nox.so
run xcd2 LWAAAI_X=0
run nox2 LWAAAI_SO=$GRAFT_REPO_ROOT/layer_wise_aaai20_amd/_lwaaai_C_nox.so
timeout -k 10 400 python scripts/op_roofline.py --all gpurun_out/op_all7.txt > gpurun_out/op_roofline7.txt 2>&1 || { tail -30 gpurun_out/op_roofline7.txt; exit 1; }
grep -A12 "per kind" gpurun_out/op_roofline7.txt
