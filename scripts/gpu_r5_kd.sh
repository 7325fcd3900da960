# round 5: the [K][C] data-gradient slabs joined to the per-step pack batch — the GPU
# suite, smoke, the default bench line, CIFAR benches and the ResNet-50 step profile
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5kd_suite.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5kd_smoke.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5kd_bench.json 2> gpurun_out/r5kd_bench.err
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5kd_cifar.jsonl 2> gpurun_out/r5kd_cifar.err
bash scripts/prof_step.sh r5kd > gpurun_out/r5kd_prof_step.txt 2>&1
