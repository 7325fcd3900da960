# round 6, call q: BN2's backward sums folded into the fused BN3 kernel (S2) — numerics, block
# tests, microbench, bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6q
timeout -k 10 400 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_block_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6q/t_bn_block.txt 2>&1
timeout -k 10 300 python -u scripts/bn3_fused_bench.py > gpurun_out/r6q/bn_fused_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6q/bench.json 2> gpurun_out/r6q/bench.err
LWAAAI_FUSE_BNBWD=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6q/bench_nofuse.json 2>> gpurun_out/r6q/bench.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6q/bench2.json 2>> gpurun_out/r6q/bench.err
