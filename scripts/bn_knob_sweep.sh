#!/bin/bash
# One gpurun call: headline bench under the BN reduce-geometry knobs (LWAAAI_BN_BLOCKS,
# LWAAAI_BN_UNROLL). Stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/knobs.txt
for cfg in "1024 4" "2048 4" "512 4" "1024 8" "2048 8"; do
  set -- $cfg
  LWAAAI_BN_BLOCKS=$1 LWAAAI_BN_UNROLL=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 6 \
    > gpurun_out/knob_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -20 gpurun_out/knob_$1_$2.log; exit 1; }
  echo "blocks=$1 unroll=$2 $(grep '^{' gpurun_out/knob_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/knobs.txt
done
