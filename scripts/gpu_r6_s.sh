# round 6, call s: step kernel traces with / without BN2's sums in the fused BN3 kernel
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/prof_step.sh r6s_s2 > /dev/null
bash scripts/prof_step.sh r6s_nos2 > /dev/null
# (the A/B used a temporary switch, LWAAAI_AB_BN2_SUMS=0, removed after the measurement)
