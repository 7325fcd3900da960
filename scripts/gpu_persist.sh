# GPU check of the persistent big-tile GEMM, the direct stem conv and the one-launch BN statistics
# finalize (all opt-in until measured): tests with them on, then bench A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export LWAAAI_GEMM_PERSIST=1 LWAAAI_STEM_DIRECT=1 LWAAAI_COLSUM_FUSED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_fused_bn_gpu.py > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 1; }
tail -2 gpurun_out/persist_tests.log
timeout -k 10 300 python scripts/stats_cost_probe.py > gpurun_out/stats_cost2.txt 2>&1 || { tail -20 gpurun_out/stats_cost2.txt; exit 1; }
cat gpurun_out/stats_cost2.txt
for cfg in "1 1 1" "0 1 1" "1 0 1" "1 1 0" "0 0 0"; do
  set -- $cfg
  LWAAAI_GEMM_PERSIST=$1 LWAAAI_STEM_DIRECT=$2 LWAAAI_COLSUM_FUSED=$3 timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bench_$1$2$3.log 2>&1 || { tail gpurun_out/bench_$1$2$3.log; exit 1; }
  echo "persist=$1 stem=$2 colsum=$3: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$1$2$3.log)"
done
timeout -k 10 400 python scripts/op_roofline.py --all gpurun_out/op_all4.txt > gpurun_out/op_roofline4.txt 2>&1 || { tail -30 gpurun_out/op_roofline4.txt; exit 1; }
