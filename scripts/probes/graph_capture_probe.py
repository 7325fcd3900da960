"""Capture one ResNet-50 training step as a HIP graph without the eager fallback (debug aid:
prints the traceback of the first call that is not capturable)."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.train.imagenet import build_trainer  # noqa: E402

tr = build_trainer("resnet50", device="cuda", compress=sys.argv[1] if len(sys.argv) > 1 else
                   "layerwise", method=sys.argv[2] if len(sys.argv) > 2 else "Topk", K=0.01,
                   graph=False)
x = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device="cuda")
t = torch.randint(0, 1000, (8,), device="cuda")
for _ in range(3):
    tr.step(x, t)
torch.cuda.synchronize()
tr.opt.device_hyper = True
tr.opt.load_hyper()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        tr._eager(x, t)
    print("capture ok")
except Exception:
    traceback.print_exc()
    sys.exit(1)
