#!/bin/bash
# One gpurun call: the BASELINE.json configs on 1 GPU (ResNet-50 compressor variants + CIFAR nets),
# then a rocprofv3 kernel trace of the headline step. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/matrix.jsonl
b() {  # name args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 400 python bench.py --steps 15 --warmup 6 "$@" > "gpurun_out/m_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/m_$name.log"; exit $rc; }
  grep '^{' "gpurun_out/m_$name.log" | tail -1 | tee -a gpurun_out/matrix.jsonl
}
b dense --compress none --method none &&
b topk_ef --ef &&
b randomk --method Randomk &&
b qsgd_entire --compress entiremodel --method RandomDithering &&
b terngrad --method TernGrad &&
b topk_entire_ef --compress entiremodel --ef &&
{ echo "=== cifar"; timeout -k 10 400 python bench_cifar.py > gpurun_out/m_cifar.log 2>&1 \
    || { tail -20 gpurun_out/m_cifar.log; exit 1; }; grep '^{' gpurun_out/m_cifar.log | tee -a gpurun_out/matrix.jsonl; } &&
{ [ "${PROFILE:-1}" = "1" ] && bash scripts/prof_step.sh final > /dev/null && tail -60 gpurun_out/final_steps.txt || true; }
echo done
