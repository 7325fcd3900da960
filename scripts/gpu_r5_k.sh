# round 5: convergence-smoke calibration sweep; step profiles with the fixed step detection
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/convergence_calibrate.py --seeds 0 --steps 600 --amp 0.15,0.3 --peak 0.05,0.1,0.2 > gpurun_out/r5k_conv_sweep.jsonl 2> gpurun_out/r5k_conv_sweep.err
bash scripts/prof_step.sh r5k > gpurun_out/r5k_prof_step.txt 2>&1
bash scripts/prof_step.sh r5k_mc --ef --ef-dense-below 4096 --momentum-correction > gpurun_out/r5k_prof_mc.txt 2>&1
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5k_prof_cifar.txt 2>&1
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 30 --warmup 8 > gpurun_out/r5k_sim8_alex.jsonl 2> gpurun_out/r5k_sim8_alex.err
