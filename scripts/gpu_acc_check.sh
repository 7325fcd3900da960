# Accuracy-half sanity: the 300-step held-out top-1 with the current kernels vs the same run with
# this session's kernel options off, and with the tuners off (fixed heuristic kernels).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python scripts/accuracy_r50.py > gpurun_out/acc_default.jsonl 2>&1 || { tail gpurun_out/acc_default.jsonl; exit 1; }
grep '^{' gpurun_out/acc_default.jsonl
LWAAAI_GEMM_PERSIST=0 LWAAAI_STEM_DIRECT=0 LWAAAI_BN_DUAL=0 LWAAAI_CONV_BIG=0 LWAAAI_BN_BLOCKS=1024 timeout -k 10 400 python scripts/accuracy_r50.py > gpurun_out/acc_oldopts.jsonl 2>&1 || { tail gpurun_out/acc_oldopts.jsonl; exit 1; }
grep '^{' gpurun_out/acc_oldopts.jsonl
LWAAAI_GEMM_TUNE=0 LWAAAI_CONV_TUNE=0 timeout -k 10 400 python scripts/accuracy_r50.py > gpurun_out/acc_notune.jsonl 2>&1 || { tail gpurun_out/acc_notune.jsonl; exit 1; }
grep '^{' gpurun_out/acc_notune.jsonl
