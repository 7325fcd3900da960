# round 5: fused passes 1/2 on the multi-task 1024-thread grid (LWAAAI_HIST12_BIG) — probe on the
# real AlexNet gradient, GPU select tests, bench A/B, AlexNet world-8 sim
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/emg
timeout -k 10 300 python -u scripts/probes/dump_em_grad.py --out /tmp/emg/em > gpurun_out/r5b2_dump.txt 2>&1
N=$(( $(stat -c %s /tmp/emg/em_g.f32) / 4 ))
for v in 1 0; do
  LWAAAI_HIST12_BIG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/b2_$v -o run --output-format csv -- build/probe/sp_v0 $N 0.01 30 0 /tmp/emg/em_g.f32 /tmp/emg/em_e.f32 > gpurun_out/r5b2_real_$v.txt 2>&1
  cp $(find /tmp/b2_$v -name '*kernel_stats.csv' | head -1) gpurun_out/r5b2_real_${v}_stats.csv
done
soft timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_mc_gpu.py tests/test_fused_sgd_gpu.py tests/test_loopback_gpu.py tests/test_topk_parity_gpu.py tests/test_ef_gpu.py tests/test_graph_step_gpu.py -q --timeout 150 --timeout-method thread > gpurun_out/r5b2_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5b2_cifar_on.jsonl 2>> gpurun_out/r5b2.err
  LWAAAI_HIST12_BIG=0 timeout -k 10 300 python -u bench_cifar.py --steps 30 --warmup 8 >> gpurun_out/r5b2_cifar_off.jsonl 2>> gpurun_out/r5b2.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5b2_r50_on.jsonl 2>> gpurun_out/r5b2.err
  LWAAAI_HIST12_BIG=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5b2_r50_off.jsonl 2>> gpurun_out/r5b2.err
done
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5b2_sim8_alex.jsonl 2>> gpurun_out/r5b2.err
