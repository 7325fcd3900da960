# round 5: PMC counters of the select chain on a real AlexNet entire-model gradient
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/emg
timeout -k 10 300 python -u scripts/probes/dump_em_grad.py --out gpurun_out/emg/em > gpurun_out/r5emp_dump.txt 2>&1
N=$(( $(stat -c %s gpurun_out/emg/em_g.f32) / 4 ))
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d /tmp/pmc1 -o run --output-format csv -- build/probe/sp_v0 $N 0.01 5 0 gpurun_out/emg/em_g.f32 gpurun_out/emg/em_e.f32 > gpurun_out/r5emp_pmc1.log 2>&1
cp $(find /tmp/pmc1 -name '*counter_collection.csv' | head -1) gpurun_out/r5emp_pmc1.csv
