# round 5: step profiles (period-detected steps), MC config profile, convergence calibration
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/prof_step.sh r5j > gpurun_out/r5j_prof_step.txt 2>&1
bash scripts/prof_step.sh r5j_mc --ef --ef-dense-below 4096 --momentum-correction > gpurun_out/r5j_prof_mc.txt 2>&1
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5j_prof_cifar.txt 2>&1
timeout -k 10 600 python -u scripts/convergence_calibrate.py --seeds 0,1 > gpurun_out/r5j_convergence_calibration.jsonl 2> gpurun_out/r5j_convergence.err
