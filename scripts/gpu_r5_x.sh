# round 5: pass-0 histogram flush contention test (8 spread copies, timing only)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2260892 9042734; do
  for v in s1 x8 x8cp2 x8s4; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/xprof_${v}_$n -o run --output-format csv -- build/probe/sp_$v $n 0.01 20 > /dev/null 2>&1
    cp $(find /tmp/xprof_${v}_$n -name '*kernel_stats.csv' | head -1) gpurun_out/r5x_${v}_${n}_stats.csv
  done
done
