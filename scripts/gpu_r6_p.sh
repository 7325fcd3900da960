# round 6, call p: round-end style records at HEAD — smoke, bench line, world-8 simulations with
# the wire priced (ResNet-50 configs, AlexNet entire-model Top-K + EF), CIFAR benches
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6p/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6p/bench.json 2> gpurun_out/r6p/bench.err
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --sim-wire --steps 15 --warmup 5 > gpurun_out/r6p/sim8_wire_r50.jsonl 2> gpurun_out/r6p/sim.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --sim-wire --steps 40 --warmup 8 > gpurun_out/r6p/sim8_wire_alexnet.jsonl 2>> gpurun_out/r6p/sim.err
timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 > gpurun_out/r6p/cifar.jsonl 2> gpurun_out/r6p/cifar.err
