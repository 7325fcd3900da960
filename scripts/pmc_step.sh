#!/bin/bash
# PMC counters of every kernel in a short bench run (two passes, each its own rocprofv3 run with
# --kernel-trace only), summarised per kernel name: wave cycles split into waiting / issue-stall /
# active, VALU and vector-memory instruction counts, and fetched bytes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcstep
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVES"
P2="FETCH_SIZE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmcs$i -o run --output-format csv -- python bench.py --steps 2 --warmup 3 --acc-steps 0 > gpurun_out/pmcstep/pass$i.log 2>&1 || exit $?
  f=$(find /tmp/pmcs$i -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" --last-step > gpurun_out/pmcstep/pass$i.txt
done
