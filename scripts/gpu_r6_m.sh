# round 6, call m: zero-padded tap kernel (no masks, immediate tap offsets) — bit-exactness vs the
# masked form, tap-vs-GEMM timing table, bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
source scripts/gpu_common.sh
soft timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "conv3_tap" > gpurun_out/r6m/t_conv.txt 2>&1
soft timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_graph_step_gpu.py > gpurun_out/r6m/t_conv_all.txt 2>&1
timeout -k 10 400 python -u scripts/conv_tap_bench.py > gpurun_out/r6m/tap_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6m/bench.json 2> gpurun_out/r6m/bench.err
