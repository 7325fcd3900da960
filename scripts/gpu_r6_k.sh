# round 6, call k: fused BN3 backward generalized to stage 2 (512 / 128 channels, two CI parts)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6k
source scripts/gpu_common.sh
soft timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py > gpurun_out/r6k/t_bn_block.txt 2>&1
timeout -k 10 300 python -u scripts/bn3_fused_bench.py > gpurun_out/r6k/bn3_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6k/bench.json 2> gpurun_out/r6k/bench.err
LWAAAI_FUSE_BN3=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6k/bench_nofuse.json 2> gpurun_out/r6k/bench_nofuse.err
