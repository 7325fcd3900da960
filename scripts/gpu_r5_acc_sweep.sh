set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# 1000-step schedule calibration for the uncompressed run
for cfg in "2.0 none" "2.0 linear" "1.0 linear" "0.5 linear"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/accuracy_r50.py --steps 1000 --methods none --seeds 0 --lr $1 --decay $2 >> gpurun_out/r5_acc_sweep.jsonl 2>> gpurun_out/r5_acc_sweep.err
done
