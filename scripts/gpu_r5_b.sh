set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mc_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5_mc_tests.txt 2>&1 || true
timeout -k 10 500 python -u -m pytest tests/test_loopback_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r5_loopback_tests.txt 2>&1 || true
LWAAAI_GRAPH_OVERLAP=0 timeout -k 10 300 python -u bench.py --simulate-world 8 --steps 10 --warmup 5 > gpurun_out/r5_sim8_r50_inline.jsonl 2> gpurun_out/r5_sim8_inline.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5_sim8_cifar.jsonl 2> gpurun_out/r5_sim8_cifar.err
LWAAAI_GRAPH_OVERLAP=0 timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5_sim8_cifar_inline.jsonl 2>> gpurun_out/r5_sim8_cifar.err
