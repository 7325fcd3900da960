set -o pipefail
mkdir -p gpurun_out
for v in "" _ns3 _ns4; do
  SO=/root/repo/layer_wise_aaai20_amd/_lwaaai_C$v.so
  echo "=== SO $v" >> gpurun_out/ns_sweep.log
  LWAAAI_SO=$SO SWEEP_TILES=2,5,6,8 timeout -k 10 300 python scripts/tile_sweep.py >> gpurun_out/ns_sweep.log 2>&1 || exit 1
done
LWAAAI_SO=/root/repo/layer_wise_aaai20_amd/_lwaaai_C_ns4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py > gpurun_out/ns4_tests.log 2>&1
