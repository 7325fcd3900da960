#!/bin/bash
# PMC counters of the stem kernels (scripts/stem_probe.py), one rocprofv3 pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcstem
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmcst$i -o run --output-format csv -- python scripts/stem_probe.py > gpurun_out/pmcstem/pass$i.log 2>&1 || exit $?
  f=$(find /tmp/pmcst$i -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" > gpurun_out/pmcstem/pass$i.txt
done
