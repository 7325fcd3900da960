# round 6, call f: exact shard dequant (uncontracted plain operators), BN dual-reduce / stem pool
# apply geometry, the 1x1 GEMM vs hipBLASLt comparison table, the bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
source scripts/gpu_common.sh
soft timeout -k 10 200 python -u scripts/probes/shard_diag.py > gpurun_out/r6f/shard_diag.txt 2>&1
soft timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_bn_gpu.py -k "dequant_shard or dual or pool or stem" > gpurun_out/r6f/t_bn.txt 2>&1
timeout -k 10 400 python -u scripts/vendor_1x1_table.py > gpurun_out/r6f/vendor_1x1.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6f/bench.json 2> gpurun_out/r6f/bench.err
LWAAAI_GRAPH_OVERLAP=comm timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_multigpu_gpu.py -k "training and Topk-layerwise-noef" > gpurun_out/r6f/t_multigpu_comm.txt 2>&1
