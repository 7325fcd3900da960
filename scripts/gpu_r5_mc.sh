# round 5: momentum-corrected first select pass, batched-load path on / off (probe binaries)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in v0 mcslow; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/mcprof_$v -o run --output-format csv -- build/probe/sp_$v 8500000 0.001 30 1 > gpurun_out/r5mc_$v.txt 2>&1
  cp $(find /tmp/mcprof_$v -name '*kernel_stats.csv' | head -1) gpurun_out/r5mc_${v}_stats.csv
done
