# 1000-step accuracy runs (stability of the accuracy half) + A/B of the BN-statistics-in-GEMM
# epilogue switches taken one at a time.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/bs_$tag.log 2>&1 || { tail gpurun_out/bs_$tag.log; exit 1; }
  echo "$tag ($*): $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bs_$tag.log)"
}
run base LWAAAI_X=0
run cross LWAAAI_CROSS_BN3=1
run bstats LWAAAI_BSTATS=1
run base2 LWAAAI_X=0
timeout -k 10 600 python scripts/accuracy_r50.py --steps 1000 > gpurun_out/acc_1000.jsonl 2>&1 || { tail gpurun_out/acc_1000.jsonl; exit 1; }
grep "^{" gpurun_out/acc_1000.jsonl
LWAAAI_GEMM_TUNE=0 LWAAAI_CONV_TUNE=0 timeout -k 10 600 python scripts/accuracy_r50.py --steps 1000 > gpurun_out/acc_1000b.jsonl 2>&1 || { tail gpurun_out/acc_1000b.jsonl; exit 1; }
grep "^{" gpurun_out/acc_1000b.jsonl
