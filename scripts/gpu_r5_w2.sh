# round 5: the bench's N > 1 path rehearsed on one box (two ranks sharing the GPU, native RCCL)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --share-gpu --backend nccl --acc-steps 50 > gpurun_out/r5w2_bench.jsonl 2> gpurun_out/r5w2_bench.err
