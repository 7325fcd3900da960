set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_base_bench.json 2> gpurun_out/r5_base_bench.err
timeout -k 10 600 bash scripts/prof_step.sh r5base
