# Stem kernels: multi-tile direct 7x7 conv, pooled-side statistics of the pool/BN backward.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_block_gpu.py tests/test_conv_gpu.py -k "stem" > gpurun_out/stem_tests.log 2>&1 || { tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 200 python scripts/stem_probe.py > gpurun_out/stem_probe.txt 2>&1 || { tail -20 gpurun_out/stem_probe.txt; exit 1; }
LWAAAI_STEM_TPW=1 timeout -k 10 200 python scripts/stem_probe.py 2>&1 | grep "stem conv" >> gpurun_out/stem_probe.txt || exit 1
LWAAAI_STEM_OCC=3 timeout -k 10 200 python scripts/stem_probe.py 2>&1 | grep "stem conv" >> gpurun_out/stem_probe.txt || exit 1
grep -v amdgpu.ids gpurun_out/stem_probe.txt
for v in "A" "B" "A2" "B2"; do
  case $v in A*) e="LWAAAI_STEM_POOLED=1";; B*) e="LWAAAI_STEM_POOLED=0 LWAAAI_STEM_TPW=1";; esac
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/stem_bench_$v.log 2>&1 || { tail -20 gpurun_out/stem_bench_$v.log; exit 1; }
  echo "$v ($e): $(grep -o '"value": [0-9.]*' gpurun_out/stem_bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem_bench_$v.log)"
done
