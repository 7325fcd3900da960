# round 5: layer-wise convergence probe (no momentum correction), sims, VGG bench, profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/probes/conv_lw_probe.py > gpurun_out/r5n_conv_lw_probe.jsonl 2> gpurun_out/r5n_conv_lw_probe.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5n_sim8_alex.jsonl 2> gpurun_out/r5n_sim8_alex.err
timeout -k 10 300 python -u bench_cifar.py --config vgg16 --steps 30 --warmup 8 > gpurun_out/r5n_bench_vgg.jsonl 2> gpurun_out/r5n_bench_vgg.err
bash scripts/prof_step.sh r5n > gpurun_out/r5n_prof_step.txt 2>&1
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5n_prof_cifar.txt 2>&1
