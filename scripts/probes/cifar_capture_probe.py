"""Bisect a HIP-graph capture problem of the CIFAR step: capture (a) forward only, (b) forward +
backward, (c) the full step, each in its own process (argv[1] = network, argv[2] = stage)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer  # noqa: E402

net, stage = sys.argv[1], sys.argv[2]
tr = CifarTrainer(net, compress="none", method="none", n_train=2048, graph=False)
for _ in range(3):
    tr.step()
torch.cuda.synchronize()
b = tr.next_batch()
x, t = b["input"].clone(), b["target"].clone()
tr.opt.device_hyper = True
tr.opt.load_hyper()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print("capturing", net, stage, flush=True)
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    if stage == "fwd":
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            out = tr.model({"input": x, "target": t})
    elif stage == "fwdbwd":
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            out = tr.ddp({"input": x, "target": t})
            loss = out["loss"].float().sum()
        loss.backward()
    else:
        tr._eager(x, t)
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed ok", net, stage, flush=True)
