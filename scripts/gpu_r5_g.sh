# round 5: alexnet sim + resnet9 bench, the 1000-step schedule sweep, then the shared-card 2-rank
# captured-training hang diagnosis (each step its own time limit; a hang ends the call)
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5g_sim8_alex.jsonl 2> gpurun_out/r5g_sim8_alex.err
timeout -k 10 300 python -u bench_cifar.py --config anchor --steps 30 --warmup 8 > gpurun_out/r5g_bench_resnet9.jsonl 2> gpurun_out/r5g_bench_resnet9.err
for cfg in "2.0 none" "1.0 linear" "0.5 linear" "0.25 linear"; do
  set -- $cfg
  timeout -k 10 400 python -u scripts/accuracy_r50.py --steps 1000 --methods none,topk0.1%+ef+mc+dense4k --seeds 0 --lr $1 --decay $2 >> gpurun_out/r5g_acc_sweep.jsonl 2>> gpurun_out/r5g_acc_sweep.err
done
T='tests/test_multigpu_gpu.py::test_training_ranks_agree_and_graph_matches_eager[Topk-layerwise-noef-2]'
LWAAAI_GRAPH_OVERLAP=1 soft timeout -k 10 150 python -u -m pytest "$T" -v --timeout 140 --timeout-method thread > gpurun_out/r5g_mgpu_overlap1.txt 2>&1
LWAAAI_GRAPH_OVERLAP=0 LWAAAI_RCCL_INIT_TIMEOUT=0 soft timeout -k 10 150 python -u -m pytest "$T" -v --timeout 140 --timeout-method thread > gpurun_out/r5g_mgpu_inline_mainthread.txt 2>&1
