# round 6, call h: weight-resident 3x3 (C = Co = 64) conv; BN3 backward fused with its GEMMs:
# unit tests, microbenches, block tests, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6h
source scripts/gpu_common.sh
soft timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "conv3_res or conv3_tap" > gpurun_out/r6h/t_conv.txt 2>&1
soft timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fused_bn_gpu.py tests/test_block_gpu.py > gpurun_out/r6h/t_bn_block.txt 2>&1
timeout -k 10 300 python -u scripts/conv3_res_bench.py > gpurun_out/r6h/res_bench.txt 2>&1
timeout -k 10 300 python -u scripts/bn3_fused_bench.py --occ > gpurun_out/r6h/bn3_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6h/bench_fused.json 2> gpurun_out/r6h/bench_fused.err
LWAAAI_FUSE_BN3=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6h/bench_nofuse.json 2> gpurun_out/r6h/bench_nofuse.err
