# round 5: pass-0 split / histogram-copy variants of the select chain, AlexNet entire-model size
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in v0 s1 s2 cp2 cp1 cp2s1 nosplit; do
    echo -n "\"$v\" " >> gpurun_out/r5u_probe.txt
    timeout -k 10 60 build/probe/sp_$v 2260892 0.01 100 >> gpurun_out/r5u_probe.txt
  done
done
for v in v0 s1 cp2s1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/uprof_$v -o run --output-format csv -- build/probe/sp_$v 2260892 0.01 20 > /dev/null 2>&1
  cp $(find /tmp/uprof_$v -name '*kernel_stats.csv' | head -1) gpurun_out/r5u_${v}_stats.csv
done
