# round 6, call n: committed state (fused BN3 / BN1 / stem backward) — full GPU suite, bench,
# step profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
source scripts/gpu_common.sh
soft timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n/pytest_gpu.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6n/bench.json 2> gpurun_out/r6n/bench.err
bash scripts/prof_step.sh r6n_r50 > /dev/null && mv gpurun_out/r6n_r50_* gpurun_out/r6n/
