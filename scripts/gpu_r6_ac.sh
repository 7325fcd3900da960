# round 6, call ac: step kernel trace at the end-of-round HEAD (re-tuned table)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/prof_step.sh r6ac > /dev/null
