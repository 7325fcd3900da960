# round 6, call z: addend chunks prefetched in the GEMM store epilogue — GEMM/block tests, bench A/B
# against a build of the previous epilogue (LWAAAI_SO) on one box, op roofline
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6z
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_block_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6z/t_gemm_block_conv.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6z/bench_pf.jsonl 2>> gpurun_out/r6z/bench.err
LWAAAI_SO=layer_wise_aaai20_amd/_exp_add0.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6z/bench_nopf.jsonl 2>> gpurun_out/r6z/bench.err
done
timeout -k 10 400 python scripts/op_roofline.py --top 40 --all gpurun_out/r6z/op_all.txt > gpurun_out/r6z/op_roofline.txt 2>&1
