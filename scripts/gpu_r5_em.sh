# round 5: the select chain on a real AlexNet entire-model gradient (dumped from an eager step)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/emg
timeout -k 10 300 python -u scripts/probes/dump_em_grad.py --out /tmp/emg/em > gpurun_out/r5em_dump.txt 2>&1
N=$(( $(stat -c %s /tmp/emg/em_g.f32) / 4 ))
for v in v0 nosplit cp2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/emprof_$v -o run --output-format csv -- build/probe/sp_$v $N 0.01 30 0 /tmp/emg/em_g.f32 /tmp/emg/em_e.f32 > gpurun_out/r5em_$v.txt 2>&1
  cp $(find /tmp/emprof_$v -name '*kernel_stats.csv' | head -1) gpurun_out/r5em_${v}_stats.csv
done
