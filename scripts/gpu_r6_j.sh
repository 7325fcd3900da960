# round 6, call j: fused BN3 backward final form — full GPU suite, bench, step profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6j
source scripts/gpu_common.sh
soft timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6j/pytest_gpu.txt 2>&1
timeout -k 10 300 python -u scripts/bn3_fused_bench.py > gpurun_out/r6j/bn3_bench.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6j/bench.json 2> gpurun_out/r6j/bench.err
bash scripts/prof_step.sh r6j_r50 > /dev/null && mv gpurun_out/r6j_r50_* gpurun_out/r6j/
