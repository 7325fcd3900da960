# Stem conv variants: occupancy target x next-tile patch prefetch.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LWAAAI_STEM_PF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "stem" > gpurun_out/stem3_tests.log 2>&1 || { tail -30 gpurun_out/stem3_tests.log; exit 1; }
tail -1 gpurun_out/stem3_tests.log
: > gpurun_out/stem3_probe.txt
for e in "LWAAAI_STEM_OCC=4" "LWAAAI_STEM_OCC=3" "LWAAAI_STEM_PF=1" "LWAAAI_STEM_PF=1 LWAAAI_STEM_OCC=3" "LWAAAI_STEM_PF=1 LWAAAI_STEM_OCC=3 LWAAAI_STEM_TPW=7" "LWAAAI_STEM_PF=1 LWAAAI_STEM_TPW=28"; do
  echo "$e: $(env $e timeout -k 10 200 python scripts/stem_probe.py 2>&1 | grep 'stem conv')" >> gpurun_out/stem3_probe.txt || exit 1
done
cat gpurun_out/stem3_probe.txt
