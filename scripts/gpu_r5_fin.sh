# round 5: step profiles at HEAD (ResNet-50 headline, VGG-16, AlexNet), default bench line
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5fin_bench.json 2> gpurun_out/r5fin_bench.err
bash scripts/prof_step.sh r5fin > gpurun_out/r5fin_prof_step.txt 2>&1
bash scripts/prof_cifar_steps.sh vgg16 alexnet > gpurun_out/r5fin_prof_cifar.txt 2>&1
