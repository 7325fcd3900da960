# round 5: fused Top-K select chain variants on the AlexNet entire-model shape (probe binaries
# built on the CPU host into build/probe, scripts/probes/select_probe.hip)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in v0 u4 u8 cp8 cp2 tpb4 split fw; do
    echo -n "\"$v\" " >> gpurun_out/r5t_probe.txt
    timeout -k 10 60 build/probe/sp_$v 9042734 0.01 100 >> gpurun_out/r5t_probe.txt
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/tprof -o run --output-format csv -- build/probe/sp_v0 9042734 0.01 20 > /dev/null 2>&1
cp $(find /tmp/tprof -name '*kernel_stats.csv' | head -1) gpurun_out/r5t_v0_stats.csv
