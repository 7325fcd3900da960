# round 5 (end): the whole GPU suite, smoke, default bench line, world-8 sims, CIFAR benches,
# ResNet-50 step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5z3_suite.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z3_smoke.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5z3_bench.json 2> gpurun_out/r5z3_bench.err
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --steps 20 --warmup 5 > gpurun_out/r5z3_sim8_r50.jsonl 2> gpurun_out/r5z3_sim8.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5z3_sim8_alex.jsonl 2>> gpurun_out/r5z3_sim8.err
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5z3_cifar.jsonl 2> gpurun_out/r5z3_cifar.err
bash scripts/prof_step.sh r5z2 > gpurun_out/r5z3_prof_step.txt 2>&1
