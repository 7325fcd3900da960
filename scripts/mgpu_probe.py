#!/usr/bin/env python
"""World-2 probe (torchrun, both ranks may share one GPU with LWAAAI_TEST_SHARE_GPU=1): train a few
HIP-graph ResNet-50 steps through the native RCCL communicator, then issue the host-side
collectives a benchmark / trainer issues after its graph replays, printing each as it completes.
usage: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 scripts/mgpu_probe.py"""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("LWAAAI_TEST_SHARE_GPU") == "1":
    os.environ["NCCL_HOSTID"] = f"lwaaai-rank{os.environ.get('RANK', '0')}"
faulthandler.dump_traceback_later(int(os.environ.get("PROBE_STACK_AFTER", "60")), exit=False)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from layer_wise_aaai20_amd.parallel import comm  # noqa: E402


def say(msg):
    print(f"[rank {os.environ.get('RANK', '?')} {time.strftime('%X')}] {msg}", flush=True)


def main():
    rank = int(os.environ["RANK"])
    dev = comm.bind_rank_device(rank)
    dist.init_process_group("nccl", device_id=dev)
    os.environ["LWAAAI_GRAPH_AUTO"] = "0"
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    torch.manual_seed(0)
    tr = build_trainer("resnet50", device=dev, compress="layerwise", method="Topk", K=0.01,
                       graph=os.environ.get("PROBE_GRAPH", "1") == "1")
    g = torch.Generator(device=dev).manual_seed(5 + rank)
    for i in range(6):
        x = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=dev, generator=g)
        t = torch.randint(0, 1000, (8,), device=dev, generator=g)
        say(f"step {i} loss {float(tr.step(x, t)):.4f} replays {tr.graph_replays}")
    torch.cuda.synchronize(dev)
    say("synchronized")
    nat = tr.ddp.engine._native
    v = torch.ones(4, device=dev)
    nat.all_reduce(v)
    torch.cuda.synchronize(dev)
    say(f"native all_reduce ok {v.tolist()}")
    dist.barrier(device_ids=[dev.index])
    say("c10d barrier ok")
    t = torch.tensor([1.0 + rank], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    say(f"c10d all_reduce ok {t.item()}")
    p = torch.cat([q.detach().float().reshape(-1) for q in tr.ddp.module.parameters()])
    parts = [torch.empty_like(p) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, p)
    torch.cuda.synchronize(dev)
    say(f"c10d all_gather ok, params equal across ranks: {torch.equal(parts[0], parts[1])}")
    del tr
    comm.shutdown_native()
    say("native shut down")
    dist.destroy_process_group()
    say("process group destroyed")
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
