# round 5: native mean cross-entropy — tests, ResNet-50 bench, step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 500 python -u -m pytest tests/test_xent_gpu.py tests/test_graph_step_gpu.py tests/test_sync_free_gpu.py tests/test_topk_parity_gpu.py tests/test_accuracy_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r5xm_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r5xm_bench.jsonl 2>> gpurun_out/r5xm.err
done
bash scripts/prof_step.sh r5xm > gpurun_out/r5xm_prof_step.txt 2>&1
