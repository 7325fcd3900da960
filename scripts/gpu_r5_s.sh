# round 5: BN backward statistics in the dgrad epilogue (A/B), AlexNet world-8 tail trace
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/sprof
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r5s_ab.jsonl 2>> gpurun_out/r5s_ab.err
  LWAAAI_BSTATS=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> gpurun_out/r5s_ab_bstats.jsonl 2>> gpurun_out/r5s_ab.err
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sprof/alex -o run --output-format csv \
  -- python bench_cifar.py --simulate-world 8 --config alexnet --steps 12 --warmup 4 > gpurun_out/r5s_alex_sim.log 2>&1
KT=$(find /tmp/sprof/alex -name '*kernel_trace.csv' | head -1)
cp "$KT" gpurun_out/r5s_alex_sim_kt.csv
