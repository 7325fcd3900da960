#!/bin/bash
# PMC counters of one conv variant (each pass its own rocprofv3 run, --kernel-trace only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
SHAPE=${SHAPE:-128,128,28,3,1,1}; ONLY=${ONLY:-fwd}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  LWAAAI_CONV_TUNE=0 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmc$i -o run --output-format csv -- python scripts/conv_variants.py --shape $SHAPE --only $ONLY --iters 10 > gpurun_out/pmc/pass$i.log 2>&1 || exit $?
  f=$(find /tmp/pmc$i -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/pmc/pass$i.csv
done
python - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for i in (1, 2):
    for r in csv.DictReader(open(f"gpurun_out/pmc/pass{i}.csv")):
        k = r["Kernel_Name"][:80]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k_gemm" not in k: continue
    print(k)
    for n, v in sorted(d.items()): print(f"   {n:28s} {v:16.0f}")
PY
