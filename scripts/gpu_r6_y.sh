# round 6, call y: step kernel trace and per-op roofline at HEAD
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
timeout -k 10 400 python scripts/op_roofline.py --top 60 --all gpurun_out/r6y/op_all.txt > gpurun_out/r6y/op_roofline.txt 2>&1
bash scripts/prof_step.sh r6y > /dev/null
