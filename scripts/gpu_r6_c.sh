# round 6, call c: the whole GPU suite after the switch pruning, the bench line, and the AlexNet /
# ResNet-50 step profiles at HEAD
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
source scripts/gpu_common.sh
soft timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6c/suite.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6c/bench.json 2> gpurun_out/r6c/bench.err
