# round 6, call e: shard-decode diagnosis, BN/stem streaming grid sweeps
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 200 python -u scripts/probes/shard_diag.py > gpurun_out/r6e/shard_diag.txt 2>&1
timeout -k 10 200 build/probe/bn_stream_probe2 > gpurun_out/r6e/bn_stream_probe2.txt 2>&1
