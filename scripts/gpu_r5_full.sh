# round 5: the whole GPU suite (as the driver runs it), smoke, MC A/B
set -e
cd $GRAFT_REPO_ROOT
source scripts/gpu_common.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
soft timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5i_gpu_suite.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5i_smoke.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 >> gpurun_out/r5i_ab_mc.jsonl 2>> gpurun_out/r5i_ab.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 --ef --ef-dense-below 4096 --momentum-correction >> gpurun_out/r5i_ab_mc.jsonl 2>> gpurun_out/r5i_ab.err
done
