# round 5: multi-rank suite after the captured-broadcast fix; the 3-seed accuracy table at the
# calibrated 1000-step schedule; CIFAR step profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 170 python -u -m pytest "tests/test_multigpu_gpu.py::test_training_ranks_agree_and_graph_matches_eager[Topk-layerwise-noef-2]" -v --timeout 160 --timeout-method thread > gpurun_out/r5h_mgpu_one.txt 2>&1
timeout -k 10 600 python -u scripts/accuracy_r50.py --steps 1000 --methods none,topk0.1%,topk0.1%+ef,topk0.1%+ef+dense4k,topk0.1%+ef+mc+dense4k --seeds 0,1,2 > gpurun_out/r5h_acc_table.jsonl 2> gpurun_out/r5h_acc_table.err
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5h_prof_cifar.txt 2>&1
soft timeout -k 10 700 python -u -m pytest tests/test_multigpu_gpu.py -v --timeout 160 --timeout-method thread > gpurun_out/r5h_mgpu_all.txt 2>&1
