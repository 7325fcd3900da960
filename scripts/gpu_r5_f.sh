# round 5: benches with the fused chain / fused SGD / zero-key histogram; then which change hangs
# the shared-card 2-rank captured training test (each step its own time limit; a hang ends the call)
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 300 python -u -m pytest tests/test_fused_sgd_gpu.py tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5f_tests_a.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err
for c in vgg16 alexnet resnet9; do
  timeout -k 10 300 python -u bench_cifar.py --config $c --steps 30 --warmup 8 >> gpurun_out/r5f_bench_cifar.jsonl 2>> gpurun_out/r5f_bench_cifar.err
done
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5f_sim8_alex.jsonl 2> gpurun_out/r5f_sim8_alex.err
T='tests/test_multigpu_gpu.py::test_training_ranks_agree_and_graph_matches_eager[Topk-layerwise-noef-2]'
LWAAAI_GRAPH_OVERLAP=1 soft timeout -k 10 150 python -u -m pytest "$T" -v --timeout 140 --timeout-method thread > gpurun_out/r5f_mgpu_overlap1.txt 2>&1
LWAAAI_GRAPH_OVERLAP=0 LWAAAI_RCCL_INIT_TIMEOUT=0 soft timeout -k 10 150 python -u -m pytest "$T" -v --timeout 140 --timeout-method thread > gpurun_out/r5f_mgpu_inline_mainthread.txt 2>&1
