# round 6, call v: tap-conv fragment addresses from hoisted byte bases + an SGPR step offset
# (LW_T3_ZSEL 2) — conv tests, tap microbench and bench, A/B against a -DLW_T3_ZSEL=1 build
# (LWAAAI_SO) on one box
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6v
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6v/t_conv.txt 2>&1
timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6v/tap_zsel2.txt 2>&1
LWAAAI_SO=layer_wise_aaai20_amd/_exp_zsel1.so timeout -k 10 300 python -u scripts/conv_tap_bench.py > gpurun_out/r6v/tap_zsel1.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6v/bench_zsel2.jsonl 2>> gpurun_out/r6v/bench.err
LWAAAI_SO=layer_wise_aaai20_amd/_exp_zsel1.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6v/bench_zsel1.jsonl 2>> gpurun_out/r6v/bench.err
done
