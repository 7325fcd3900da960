# round 6, call ab: re-tune every kernel choice from scratch after this round's kernel changes and
# A/B the new table against the shipped one on one box
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
echo '{}' > /tmp/tune_fresh.json
LWAAAI_TUNE_FILE=/tmp/tune_fresh.json timeout -k 10 600 python -u bench.py --steps 10 --warmup 5 > gpurun_out/r6ab/bench_tuning.json 2> gpurun_out/r6ab/bench.err
cp /tmp/tune_fresh.json gpurun_out/r6ab/tune_fresh.json
for i in 1 2; do
LWAAAI_TUNE_FILE=/tmp/tune_fresh.json timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6ab/bench_fresh.jsonl 2>> gpurun_out/r6ab/bench.err
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6ab/bench_shipped.jsonl 2>> gpurun_out/r6ab/bench.err
done
