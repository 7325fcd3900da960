# round 5: pass 0 on 1024-thread multi-task workgroups (LW_HIST0_BIG_MIN) vs the 256-thread grid,
# synthetic sizes + the real AlexNet entire-model gradient; payload hashes must match
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/emg
timeout -k 10 300 python -u scripts/probes/dump_em_grad.py --out /tmp/emg/em > gpurun_out/r5b0_dump.txt 2>&1
N=$(( $(stat -c %s /tmp/emg/em_g.f32) / 4 ))
for v in v0 small0; do
  for n in 2260892 9042734 25557032; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/b0_${v}_$n -o run --output-format csv -- build/probe/sp_$v $n 0.01 30 > gpurun_out/r5b0_${v}_$n.txt 2>&1
    cp $(find /tmp/b0_${v}_$n -name '*kernel_stats.csv' | head -1) gpurun_out/r5b0_${v}_${n}_stats.csv
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/b0_${v}_mc -o run --output-format csv -- build/probe/sp_$v 8500000 0.001 30 1 > gpurun_out/r5b0_${v}_mc.txt 2>&1
  cp $(find /tmp/b0_${v}_mc -name '*kernel_stats.csv' | head -1) gpurun_out/r5b0_${v}_mc_stats.csv
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/b0_${v}_real -o run --output-format csv -- build/probe/sp_$v $N 0.01 30 0 /tmp/emg/em_g.f32 /tmp/emg/em_e.f32 > gpurun_out/r5b0_${v}_real.txt 2>&1
  cp $(find /tmp/b0_${v}_real -name '*kernel_stats.csv' | head -1) gpurun_out/r5b0_${v}_real_stats.csv
done
