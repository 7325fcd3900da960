# round 6, call o: XOR-swizzled M/N-contiguous GEMM tiles (conflict-free transposing reads) — GEMM /
# conv tests, bench, PMC pass on the weight-gradient GEMMs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
source scripts/gpu_common.sh
soft timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_block_gpu.py tests/test_mf32_gpu.py tests/test_fp16_gpu.py > gpurun_out/r6o/t_gemm_conv.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6o/bench.json 2> gpurun_out/r6o/bench.err
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
for cfg in "256 256 14 wgrad_tuned" "64 64 56 wgrad_tuned"; do
  set -- $cfg
  tag=c$1_h$3_$4
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmc_$tag$i -o run --output-format csv -- python scripts/tap_one.py --c $1 --co $2 --hw $3 --pass $4 --iters 5 > gpurun_out/r6o/$tag.$i.log 2>&1 || exit $?
    f=$(find /tmp/pmc_$tag$i -name '*counter_collection.csv' | head -1)
    cp "$f" gpurun_out/r6o/$tag.$i.csv
  done
  python scripts/pmc_summ.py gpurun_out/r6o/$tag.1.csv gpurun_out/r6o/$tag.2.csv > gpurun_out/r6o/$tag.txt
done
echo pmc-done
