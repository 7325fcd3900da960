# Same-box A/B of the stem conv defaults: prefetch at 3 waves/SIMD (A) vs no prefetch at 4 (B).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in A B A2 B2; do
  case $v in A*) e="LWAAAI_STEM_PF=1";; B*) e="LWAAAI_STEM_PF=0 LWAAAI_STEM_OCC=4";; esac
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/stem5_bench_$v.log 2>&1 || { tail -20 gpurun_out/stem5_bench_$v.log; exit 1; }
  echo "$v ($e): $(grep -o '"value": [0-9.]*' gpurun_out/stem5_bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem5_bench_$v.log)"
done
