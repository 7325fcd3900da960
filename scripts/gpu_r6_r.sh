# round 6, call r: A/B of BN2's sums in the fused BN3 kernel (stage 1 only), alternating on one box
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
timeout -k 10 300 python -u -m pytest tests/test_block_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6r/t_block.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6r/bench_s2.jsonl 2>> gpurun_out/r6r/bench.err
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6r/bench_nos2.jsonl 2>> gpurun_out/r6r/bench.err
done
