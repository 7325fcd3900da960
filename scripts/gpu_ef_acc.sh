#!/bin/bash
# EF root-cause experiments (CIFAR ResNet-9 dawn recipe, scripts/ef_trace.py) and the ResNet-50
# 1000-step accuracy reference points over 3 seeds (scripts/accuracy_r50.py). Each step under its
# own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in ${EF_STEPS:-table trace acc}; do
  case $step in
    table) timeout -k 10 900 python -u scripts/ef_trace.py > gpurun_out/ef_table.jsonl 2> gpurun_out/ef_table.err || exit $? ;;
    trace) timeout -k 10 600 python -u scripts/ef_trace.py --only 2,3,5 --every 50 \
             --trace-out gpurun_out/ef_trace.jsonl > gpurun_out/ef_trace_summary.jsonl 2> gpurun_out/ef_trace.err || exit $? ;;
    acc) timeout -k 10 900 python -u scripts/accuracy_r50.py --steps 1000 --seeds 0,1,2 \
           --methods none,topk0.1%,topk0.1%+ef,topk0.1%+ef+mc+dense4k > gpurun_out/acc_1000.jsonl 2> gpurun_out/acc_1000.err || exit $? ;;
  esac
  echo "step $step done"
done
