cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
for sh in 64,64,56,3,1,1 128,128,28,3,1,1 256,256,14,3,1,1 512,512,7,3,1,1; do
  timeout -k 10 120 python scripts/conv_variants.py --shape $sh >> gpurun_out/variants.log 2>&1 || exit $?
done
cat gpurun_out/variants.log
