#!/bin/bash
# A/B of env-switched variants of the 1-GPU bench in one call: VARIANTS="A=1,B=0 A=0,B=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in $VARIANTS; do
  envs=$(echo $v | tr ',' ' ')
  echo "=== $v" >> gpurun_out/ab.log
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-8} ${BENCH_ARGS:-} >> gpurun_out/ab.log 2>&1 || exit $?
done
grep -E "^===|\"value\"" gpurun_out/ab.log | sed -E 's/.*"value": ([0-9.]+).*"ms_per_step": ([0-9.]+).*/  \1 img\/s  \2 ms/'
