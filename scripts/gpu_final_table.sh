#!/bin/bash
# Regenerate the shipped gfx950 tuning table (ops/tune_gfx950.json) from scratch and the accuracy
# reference points measured with it pinned. One gpurun call; each step under its own time limit,
# stop at the first failure. Afterwards (CPU): cp gpurun_out/tune_final.json
# layer_wise_aaai20_amd/ops/tune_gfx950.json and scripts/acc_reference.py gpurun_out/acc_final.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/tune_final.json
export LWAAAI_TUNE_FILE=gpurun_out/tune_final.json
STEPS="tb:420:python -u bench.py;;tc:300:python -u bench_cifar.py --config all;;\
acc:600:python -u scripts/accuracy_r50.py --steps 1000 --seeds 0,1,2 \
--methods none,topk0.1%,topk0.1%+ef,topk0.1%+ef+dense4k,topk0.1%+ef+mc+dense4k \
> gpurun_out/acc_final.jsonl" bash scripts/gpu_steps.sh
