# 1000-step schedule calibration: the uncompressed run and the strongest
# compressed variant (momentum correction) under each candidate schedule, seed 0
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "2.0 none" "1.0 linear" "0.5 linear" "0.25 linear"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/accuracy_r50.py --steps 1000 --methods none,topk0.1%+ef+mc+dense4k --seeds 0 --lr $1 --decay $2 >> gpurun_out/r5_acc_sweep.jsonl 2>> gpurun_out/r5_acc_sweep.err
done
