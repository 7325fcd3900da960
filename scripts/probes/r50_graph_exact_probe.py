"""ResNet-50 (fused MFMA path) graph vs eager: max |param| difference after each step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.train.imagenet import build_trainer  # noqa: E402

method, mode = sys.argv[1], sys.argv[2]
g = torch.Generator(device="cuda").manual_seed(3)
data = [(torch.randint(0, 256, (16, 96, 96, 3), dtype=torch.uint8, device="cuda", generator=g),
         torch.randint(0, 1000, (16,), device="cuda", generator=g)) for _ in range(int(os.environ.get("PROBE_STEPS", "8")))]
runs = {}
for graph in (False, True):
    torch.manual_seed(0)
    tr = build_trainer("resnet50", device="cuda", compress=mode, method=method, K=0.01,
                       error_feedback=True, graph=graph)
    hist = []
    for x, t in data:
        tr.step(x, t)
        torch.cuda.synchronize()
        hist.append(torch.cat([p.detach().float().reshape(-1) for p in tr.ddp.module.parameters()]))
    runs[graph] = hist
print(method, mode, "max |dparam| per step:",
      ["%.1e" % float((a - b).abs().max()) for a, b in zip(runs[False], runs[True])], flush=True)
