# round 6, call t: a2-free forward (conv3 applies BN2 in its prologue, the fused BN3 backward
# re-forms a2 from c2) — numerics, block tests, A/B on one box, tuning-table entries, step trace
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6t
timeout -k 10 400 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_block_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6t/t_bn_block.txt 2>&1
cp layer_wise_aaai20_amd/ops/tune_gfx950.json /tmp/tune_new.json
LWAAAI_TUNE_FILE=/tmp/tune_new.json timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 > gpurun_out/r6t/bench_tune.json 2> gpurun_out/r6t/bench.err
cp /tmp/tune_new.json gpurun_out/r6t/tune_new.json
for i in 1 2; do
LWAAAI_TUNE_FILE=/tmp/tune_new.json timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6t/bench_a2free.jsonl 2>> gpurun_out/r6t/bench.err
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 >> gpurun_out/r6t/bench_a2.jsonl 2>> gpurun_out/r6t/bench.err
done
# (the A/B's second arm ran with a temporary switch, LWAAAI_AB_A2FREE=0, removed afterwards)
