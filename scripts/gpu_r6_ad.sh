# round 6, call ad: BN=64 tap-conv masking by max() with per-lane penalties (LW_T3_PEN) — conv
# tests, tap microbench and bench, A/B against a -DLW_T3_PEN=0 build (LWAAAI_SO) on one box
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ad
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_block_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6ad/t_conv_block.txt 2>&1
timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6ad/tap_pen1.txt 2>&1
LWAAAI_SO=layer_wise_aaai20_amd/_exp_pen0.so timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6ad/tap_pen0.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6ad/bench_pen1.jsonl 2>> gpurun_out/r6ad/bench.err
LWAAAI_SO=layer_wise_aaai20_amd/_exp_pen0.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6ad/bench_pen0.jsonl 2>> gpurun_out/r6ad/bench.err
done
