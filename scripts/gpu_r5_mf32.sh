set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mf32_gpu.py tests/test_mc_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5_mf32_tests.txt 2>&1 || true
timeout -k 10 700 python -u scripts/mf32_ab.py --rounds 2 > gpurun_out/r5_mf32_ab.txt 2>&1
