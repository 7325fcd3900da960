# round 6, call d: the tests the switch pruning touched, the real 2-rank RCCL training tests on the
# quantised reduce-scatter wire (default inline exchange), and one diagnostic of the side-branch
# mode under a real communicator
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
source scripts/gpu_common.sh
soft timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_fused_sgd_gpu.py tests/test_topk_parity_gpu.py -k "pack_dgrad_nkc or fused_sgd or claimed or topk_bit_exact" > gpurun_out/r6d/t_fix.txt 2>&1
soft timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "dequant_shard" > gpurun_out/r6d/t_shard.txt 2>&1
soft timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_multigpu_gpu.py -k "training and (qrs or RandomDithering or Topk-layerwise-noef)" > gpurun_out/r6d/t_multigpu.txt 2>&1
LWAAAI_GRAPH_OVERLAP=1 soft timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_multigpu_gpu.py -k "training and Topk-layerwise-noef" > gpurun_out/r6d/t_multigpu_overlap1.txt 2>&1
