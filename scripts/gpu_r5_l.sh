# round 5: convergence calibration at the chosen settings (3 seeds); world-8 simulations of
# BASELINE configs 3-5 (alternating windows); step profiles
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/convergence_calibrate.py --seeds 0,1,2 > gpurun_out/r5l_convergence_calibration.jsonl 2> gpurun_out/r5l_conv.err
timeout -k 10 500 python -u bench.py --simulate-world 8 --sim-all --steps 20 --warmup 5 > gpurun_out/r5l_sim8_r50.jsonl 2> gpurun_out/r5l_sim8.err
timeout -k 10 300 python -u bench_cifar.py --simulate-world 8 --config alexnet --steps 60 --warmup 8 > gpurun_out/r5l_sim8_alex.jsonl 2>> gpurun_out/r5l_sim8.err
bash scripts/prof_step.sh r5l > gpurun_out/r5l_prof_step.txt 2>&1
bash scripts/prof_step.sh r5l_mc --ef --ef-dense-below 4096 --momentum-correction > gpurun_out/r5l_prof_mc.txt 2>&1
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5l_prof_cifar.txt 2>&1
