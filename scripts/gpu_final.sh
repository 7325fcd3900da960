# Final round: the full GPU round (suite, smoke, bench, profile, CIFAR, share2), then the stem
# conv variant probe.
cd $GRAFT_REPO_ROOT
bash scripts/gpu_full.sh || exit 1
bash scripts/gpu_stem3.sh
