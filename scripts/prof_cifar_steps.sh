#!/bin/bash
# Steady-state per-step kernel breakdown of the CIFAR benches (one rocprofv3 kernel trace per
# config; scripts/trace_steps.py keeps only the last 5 steps, so warm-up, tuning and graph capture
# are excluded). usage: scripts/prof_cifar_steps.sh [configs]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cifar_steps /tmp/cprof
for c in ${@:-anchor vgg16 alexnet}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cprof/$c -o run --output-format csv \
    -- python bench_cifar.py --config $c --steps 12 --warmup 8 > gpurun_out/cifar_steps/$c.log 2>&1 || exit $?
  KT=$(find /tmp/cprof/$c -name '*kernel_trace.csv' | head -1)
  SEQ=gpurun_out/cifar_steps/${c}_seq.txt python scripts/trace_steps.py "$KT" 5 -v > gpurun_out/cifar_steps/${c}_steps.txt || exit $?
  head -3 gpurun_out/cifar_steps/${c}_steps.txt
done
