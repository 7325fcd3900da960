# Bench A/B over BN reduce / statistics-fold geometry switches (env only, same build).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/ab_$tag.log 2>&1 || { tail gpurun_out/ab_$tag.log; exit 1; }
  echo "$tag ($*): $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/ab_$tag.log)"
}
run base LWAAAI_X=0
run colsum256 LWAAAI_COLSUM_BLOCKS=256
run colsum64 LWAAAI_COLSUM_BLOCKS=64
run bn512 LWAAAI_BN_BLOCKS=512
run bn2048 LWAAAI_BN_BLOCKS=2048
run base2 LWAAAI_X=0
