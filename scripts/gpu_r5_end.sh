# round 5 (end, HEAD): smoke, the default bench line, world-8 sims, CIFAR benches
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5end_smoke.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5end_bench.json 2> gpurun_out/r5end_bench.err
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --steps 20 --warmup 5 > gpurun_out/r5end_sim8_r50.jsonl 2> gpurun_out/r5end_sim8.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5end_sim8_alex.jsonl 2>> gpurun_out/r5end_sim8.err
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r5end_cifar.jsonl 2> gpurun_out/r5end_cifar.err
