#!/bin/bash
# rocprofv3 counter passes over the tap-reuse conv kernels (one pass per counter set)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tap
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
for pas in fwd wgrad; do
  timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/pmc_tap/$pas -o run \
    --output-format csv -- python scripts/tap_one.py --pass $pas --iters 10 || exit $?
done
echo pmc-done
