# round 5: per-step pack batch A/B on one box (LWAAAI_KC_BATCH=0 / 1 alternating)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for kb in 0 1; do
    echo "kc_batch=$kb" >> gpurun_out/r5kcab.jsonl
    LWAAAI_KC_BATCH=$kb timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5kcab.jsonl 2>> gpurun_out/r5kcab.err
  done
done
