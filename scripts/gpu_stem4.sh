# Stem conv default = next-tile prefetch at 3 waves/SIMD: tests, probe (tiles per workgroup), bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_block_gpu.py -k "stem" > gpurun_out/stem4_tests.log 2>&1 || { tail -30 gpurun_out/stem4_tests.log; exit 1; }
tail -1 gpurun_out/stem4_tests.log
: > gpurun_out/stem4_probe.txt
for e in "LWAAAI_STEM_TPW=0" "LWAAAI_STEM_TPW=28" "LWAAAI_STEM_TPW=20"; do
  echo "$e: $(env $e timeout -k 10 200 python scripts/stem_probe.py 2>&1 | grep 'stem conv')" >> gpurun_out/stem4_probe.txt || exit 1
done
cat gpurun_out/stem4_probe.txt
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/stem4_bench_$v.log 2>&1 || { tail -20 gpurun_out/stem4_bench_$v.log; exit 1; }
  echo "bench $v: $(grep -o '"value": [0-9.]*' gpurun_out/stem4_bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem4_bench_$v.log)"
done
