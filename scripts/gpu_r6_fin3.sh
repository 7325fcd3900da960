# round 6, final record at HEAD after the 64-channel tap masking change: whole GPU suite, smoke, bench line, world-8 wire-priced sims, CIFAR
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6fin3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6fin3/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6fin3/bench.json 2> gpurun_out/r6fin3/bench.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6fin3/pytest_gpu.txt 2>&1
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --sim-wire --steps 15 --warmup 5 > gpurun_out/r6fin3/sim8_wire_r50.jsonl 2> gpurun_out/r6fin3/sim.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --sim-wire --steps 40 --warmup 8 > gpurun_out/r6fin3/sim8_wire_alexnet.jsonl 2>> gpurun_out/r6fin3/sim.err
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r6fin3/cifar.jsonl 2> gpurun_out/r6fin3/cifar.err
