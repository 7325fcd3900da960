# round 5: quarter-task write verification; which layer-wise settings learn the smoke task
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py tests/test_mc_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5m_tests.txt 2>&1
timeout -k 10 600 python -u scripts/probes/conv_lw_probe.py > gpurun_out/r5m_conv_lw_probe.jsonl 2> gpurun_out/r5m_conv_lw_probe.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5m_sim8_alex.jsonl 2> gpurun_out/r5m_sim8_alex.err
timeout -k 10 300 python -u bench_cifar.py --config vgg16 --steps 30 --warmup 8 > gpurun_out/r5m_bench_vgg.jsonl 2> gpurun_out/r5m_bench_vgg.err
