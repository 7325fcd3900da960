# Full GPU round: GPU suite, smoke, 1-GPU bench, rocprofv3 step breakdown, CIFAR configs.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_pytest.log 2>&1 || { tail -40 gpurun_out/full_pytest.log; exit 1; }
tail -3 gpurun_out/full_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -2 gpurun_out/full_smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 8 > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log
timeout -k 10 900 bash scripts/prof_step.sh r4_final --acc-steps 0 > gpurun_out/full_prof.log 2>&1 || { tail -20 gpurun_out/full_prof.log; exit 1; }
head -3 gpurun_out/r4_final_steps.txt
timeout -k 10 600 python bench_cifar.py --config all > gpurun_out/full_cifar.log 2>&1 || { tail -20 gpurun_out/full_cifar.log; exit 1; }
grep -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/full_cifar.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 2 --batch 64 --share-gpu --backend gloo --acc-steps 0 > gpurun_out/full_share2.log 2>&1 || { tail -20 gpurun_out/full_share2.log; exit 1; }
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*' gpurun_out/full_share2.log
