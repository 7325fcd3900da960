# round 5: MC bitwise fix, new multi-rank cases, overlap-mode A/B under simulated world 8
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_mc_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_multigpu_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r5c_tests.txt 2>&1 || true
for m in comm 1 0; do
  LWAAAI_GRAPH_OVERLAP=$m timeout -k 10 400 python -u bench.py --simulate-world 8 --sim-all --steps 10 --warmup 5 > gpurun_out/r5c_sim8_r50_$m.jsonl 2> gpurun_out/r5c_sim8_r50_$m.err
  LWAAAI_GRAPH_OVERLAP=$m timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5c_sim8_alex_$m.jsonl 2> gpurun_out/r5c_sim8_alex_$m.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c_prof_alex -o alex -- python bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5c_prof_alex.log 2>&1
