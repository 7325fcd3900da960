cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py tests/test_gemm_gpu.py tests/test_conv_gpu.py > gpurun_out/bn_tests.log 2>&1 || { tail -30 gpurun_out/bn_tests.log; exit 1; }
tail -2 gpurun_out/bn_tests.log
timeout -k 10 300 python scripts/stats_cost_probe.py > gpurun_out/stats_cost.txt 2>&1 || { tail -20 gpurun_out/stats_cost.txt; exit 1; }
cat gpurun_out/stats_cost.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bench_dual.log 2>&1 || { tail gpurun_out/bench_dual.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench_dual.log
LWAAAI_BN_DUAL=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bench_nodual.log 2>&1 || { tail gpurun_out/bench_nodual.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench_nodual.log
