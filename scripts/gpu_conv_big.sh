cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 400 python scripts/op_roofline.py --all gpurun_out/op_all.txt --blas > gpurun_out/op_roofline3.txt 2>&1 || { tail -30 gpurun_out/op_roofline3.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bench3.log 2>&1 || { tail gpurun_out/bench3.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench3.log
