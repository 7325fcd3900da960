# round 6, call i: fused BN3 backward — dual (downsample) form, two tiles of loads in flight
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6i
source scripts/gpu_common.sh
soft timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py > gpurun_out/r6i/t_bn_block.txt 2>&1
timeout -k 10 300 python -u scripts/bn3_fused_bench.py --depth > gpurun_out/r6i/bn3_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6i/bench_fused.json 2> gpurun_out/r6i/bench_fused.err
LWAAAI_FUSE_BN3=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6i/bench_nofuse.json 2> gpurun_out/r6i/bench_nofuse.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6i/bench_fused2.json 2> gpurun_out/r6i/bench_fused2.err
