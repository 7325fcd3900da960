# Stem / ReLU-pool backward geometry: one row per thread in the apply passes, 4-row reduce loop.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_block_gpu.py tests/test_conv_gpu.py tests/test_fused_bn_gpu.py > gpurun_out/stem2_tests.log 2>&1 || { tail -30 gpurun_out/stem2_tests.log; exit 1; }
tail -1 gpurun_out/stem2_tests.log
timeout -k 10 200 python scripts/stem_probe.py > gpurun_out/stem2_probe.txt 2>&1 || { tail -20 gpurun_out/stem2_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stem2_probe.txt
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/stem2_bench_$v.log 2>&1 || { tail -20 gpurun_out/stem2_bench_$v.log; exit 1; }
  echo "bench $v: $(grep -o '"value": [0-9.]*' gpurun_out/stem2_bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem2_bench_$v.log)"
done
timeout -k 10 300 python bench_cifar.py --config all > gpurun_out/stem2_cifar.log 2>&1 || { tail -20 gpurun_out/stem2_cifar.log; exit 1; }
grep -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/stem2_cifar.log
