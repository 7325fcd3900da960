# A/B: split-K exploration for weight gradients (tuner picks (tile, splits)); GEMM/conv/block tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py > gpurun_out/splits_tests.log 2>&1 || { tail -30 gpurun_out/splits_tests.log; exit 1; }
tail -2 gpurun_out/splits_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bench_sk$i.log 2>&1 || { tail gpurun_out/bench_sk$i.log; exit 1; }
echo "run $i: $(grep -o '"value": [0-9.]*' gpurun_out/bench_sk$i.log)"
done
timeout -k 10 400 python scripts/op_roofline.py --all gpurun_out/op_all5.txt > gpurun_out/op_roofline5.txt 2>&1 || { tail -30 gpurun_out/op_roofline5.txt; exit 1; }
grep -A12 "per kind" gpurun_out/op_roofline5.txt
