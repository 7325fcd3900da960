# round 5: select chain with batched loads; pass-0 split variants at three entire-model sizes
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for n in 2260892 9042734 25557032; do
    for v in v0 s1 s2 nosplit; do
      echo -n "\"$v\" " >> gpurun_out/r5w_probe.txt
      timeout -k 10 60 build/probe/sp_$v $n 0.01 100 >> gpurun_out/r5w_probe.txt
    done
  done
done
for v in v0 s1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/wprof_$v -o run --output-format csv -- build/probe/sp_$v 2260892 0.01 20 > /dev/null 2>&1
  cp $(find /tmp/wprof_$v -name '*kernel_stats.csv' | head -1) gpurun_out/r5w_${v}_stats.csv
done
