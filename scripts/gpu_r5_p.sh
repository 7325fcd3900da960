# round 5: fused MC + claimed overwrite tests, convergence smoke, MC vs plain A/B, multi-rank suite
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 400 python -u -m pytest tests/test_mc_gpu.py tests/test_fused_sgd_gpu.py tests/test_kernels_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5p_tests.txt 2>&1
soft timeout -k 10 500 python -u -m pytest tests/test_convergence_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/r5p_convergence.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5p_ab_mc.jsonl 2>> gpurun_out/r5p_ab.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 --ef --ef-dense-below 4096 --momentum-correction >> gpurun_out/r5p_ab_mc.jsonl 2>> gpurun_out/r5p_ab.err
done
soft timeout -k 10 600 python -u -m pytest tests/test_multigpu_gpu.py -q --timeout 160 --timeout-method thread > gpurun_out/r5p_mgpu.txt 2>&1
