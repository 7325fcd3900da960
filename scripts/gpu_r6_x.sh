# round 6, call x: register-staged GEMM K loop unrolled by two (LW_KLOOP2) — GEMM/conv/block
# tests, conv microbench, counters and bench, A/B against a -DLW_KLOOP2=0 build (LWAAAI_SO)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6x
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_gemm_gpu.py tests/test_block_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6x/t_conv_gemm_block.txt 2>&1
timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6x/tap_kl2.txt 2>&1
LWAAAI_SO=layer_wise_aaai20_amd/_exp_kl1.so timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6x/tap_kl1.txt 2>&1
P="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/r6x/pmc_kl2 -o run --output-format csv -- python scripts/tap_one.py --c 256 --co 256 --hw 14 --pass wgrad_tuned --iters 5 > /dev/null 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6x/bench_kl2.jsonl 2>> gpurun_out/r6x/bench.err
LWAAAI_SO=layer_wise_aaai20_amd/_exp_kl1.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6x/bench_kl1.jsonl 2>> gpurun_out/r6x/bench.err
done
