# round 6, call b: new wire / kernel tests, the bench line with the BN apply grids, and the
# wire-priced world-8 simulations for the overlap-mode decision
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
source scripts/gpu_common.sh
soft timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "dequant_shard or wire_wait or splitk_discard" > gpurun_out/r6b/t_kernels.txt 2>&1
soft timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_loopback_gpu.py > gpurun_out/r6b/t_loopback.txt 2>&1
soft timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_multigpu_gpu.py -k "qrs or RandomDithering" > gpurun_out/r6b/t_multigpu.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err
for ov in 0 1 comm; do
  timeout -k 10 400 python -u bench.py --simulate-world 8 --sim-all --sim-wire --sim-overlap $ov --steps 15 --warmup 5 >> gpurun_out/r6b/sim8_wire_r50.jsonl 2>> gpurun_out/r6b/sim.err
done
for ov in 0 1 comm; do
  timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --sim-wire --sim-overlap $ov --steps 40 --warmup 8 >> gpurun_out/r6b/sim8_wire_alexnet.jsonl 2>> gpurun_out/r6b/sim.err
done
