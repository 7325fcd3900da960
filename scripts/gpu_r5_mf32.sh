set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mf32_gpu.py tests/test_mc_gpu.py tests/test_loopback_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r5_mf32_tests.txt 2>&1 || true
timeout -k 10 500 python -u scripts/mf32_ab.py --rounds 2 > gpurun_out/r5_mf32_ab.txt 2>&1 || true
timeout -k 10 400 python -u bench.py --simulate-world 8 --sim-all --steps 10 --warmup 5 > gpurun_out/r5_sim8_r50.jsonl 2> gpurun_out/r5_sim8_r50.err
