#!/bin/bash
# Counter passes (one rocprofv3 run each, --kernel-trace only) over one GEMM problem:
#   bash scripts/pmc_gemm.sh TAG M N K TILE [LAYOUT]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/pmc_$TAG
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmcg$TAG$i -o run --output-format csv -- python scripts/gemm_one.py "$@" > gpurun_out/pmc_$TAG/pass$i.log 2>&1 || exit $?
  f=$(find /tmp/pmcg$TAG$i -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" > gpurun_out/pmc_$TAG/pass$i.txt
done
timeout -k 5 60 python scripts/gemm_one.py "$@" > gpurun_out/pmc_$TAG/time.txt 2>&1
