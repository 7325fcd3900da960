# A/B: 3-stage LDS-DMA ring in the tiled GEMM (build -DLW_NSTAGE=3, _lwaaai_C_ns3.so) vs 2 stages.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 --acc-steps 0 > gpurun_out/ns_$tag.log 2>&1 || { tail gpurun_out/ns_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/ns_$tag.log)"
}
run ns2 LWAAAI_X=0
run ns3 LWAAAI_SO=$GRAFT_REPO_ROOT/layer_wise_aaai20_amd/_lwaaai_C_ns3.so
run ns2b LWAAAI_X=0
run ns3b LWAAAI_SO=$GRAFT_REPO_ROOT/layer_wise_aaai20_amd/_lwaaai_C_ns3.so
