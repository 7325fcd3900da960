# round 6, call w: interleaved B-gather chunk stores (LW_BGATHER_IL) in the weight-gradient convs —
# conv/GEMM tests, wgrad microbench, LDS-conflict counters and bench, A/B against a
# -DLW_BGATHER_IL=0 build (LWAAAI_SO) on one box
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6w/t_conv_gemm.txt 2>&1
timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6w/tap_il1.txt 2>&1
LWAAAI_SO=layer_wise_aaai20_amd/_exp_il0.so timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6w/tap_il0.txt 2>&1
P="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/r6w/pmc_il1 -o run --output-format csv -- python scripts/tap_one.py --c 256 --co 256 --hw 14 --pass wgrad_tuned --iters 5 > /dev/null 2>&1
LWAAAI_SO=layer_wise_aaai20_amd/_exp_il0.so timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/r6w/pmc_il0 -o run --output-format csv -- python scripts/tap_one.py --c 256 --co 256 --hw 14 --pass wgrad_tuned --iters 5 > /dev/null 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6w/bench_il1.jsonl 2>> gpurun_out/r6w/bench.err
LWAAAI_SO=layer_wise_aaai20_amd/_exp_il0.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6w/bench_il0.jsonl 2>> gpurun_out/r6w/bench.err
done
