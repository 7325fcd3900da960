# Direct 3x3 conv (layer-1) tests + timing probe + bench A/B; BN reduce blocks 512 vs 1024.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_fused_bn_gpu.py > gpurun_out/d3_tests.log 2>&1 || { tail -30 gpurun_out/d3_tests.log; exit 1; }
tail -2 gpurun_out/d3_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/d3_$tag.log 2>&1 || { tail gpurun_out/d3_$tag.log; exit 1; }
  echo "$tag ($*): $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/d3_$tag.log)"
}
run default LWAAAI_X=0
run nodirect3 LWAAAI_CONV3_DIRECT=0
run bn1024 LWAAAI_BN_BLOCKS=1024
run bn384 LWAAAI_BN_BLOCKS=384
run default2 LWAAAI_X=0
timeout -k 10 400 python scripts/op_roofline.py --all gpurun_out/op_all6.txt > gpurun_out/op_roofline6.txt 2>&1 || { tail -30 gpurun_out/op_roofline6.txt; exit 1; }
grep "x(256, 64, 56, 56) w(64, 64, 3, 3)" gpurun_out/op_all6.txt | head -12
