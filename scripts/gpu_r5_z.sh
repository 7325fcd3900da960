# round 5: single-launch entire-model select (k_select_persist) vs the launch chain: bitwise
# payload / residual hashes and timing at three sizes
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2260892 4000000 9042734; do
  LWAAAI_SELECT_PERSIST=0 timeout -k 10 60 build/probe/sp_v0 $n 0.01 50 > gpurun_out/r5za_chain_$n.txt
  timeout -k 10 60 build/probe/sp_v0 $n 0.01 50 > gpurun_out/r5za_persist_$n.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/zaprof -o run --output-format csv -- build/probe/sp_v0 2260892 0.01 20 > /dev/null 2>&1
cp $(find /tmp/zaprof -name '*kernel_stats.csv' | head -1) gpurun_out/r5za_persist_stats.csv
