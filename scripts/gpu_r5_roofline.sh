set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/op_roofline.py --top 70 --all gpurun_out/r5_op_all.txt > gpurun_out/r5_op_roofline.txt 2>&1
timeout -k 10 400 bash scripts/prof_step.sh r5base224
