#!/usr/bin/env python
"""One tap-reuse conv shape, run N times (for rocprofv3 counter passes).
usage: python scripts/tap_one.py [--n 256 --c 128 --co 128 --hw 28 --pass fwd|dgrad|wgrad|wgrad_tuned|fwd_tuned --iters 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--c", type=int, default=128)
ap.add_argument("--co", type=int, default=128)
ap.add_argument("--hw", type=int, default=28)
ap.add_argument("--pass", dest="pas", default="fwd")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
lib = load()
CL = torch.channels_last
x = torch.randn(a.n, a.c, a.hw, a.hw, device="cuda").bfloat16().contiguous(memory_format=CL)
w = (torch.randn(a.co, a.c, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
dy = torch.randn(a.n, a.co, a.hw, a.hw, device="cuda").bfloat16().contiguous(memory_format=CL)
op, _, _ = CV.pack_fwd_weight(w)
wf = CV.tap_dgrad_weight(w)
dw = torch.zeros(a.co, a.c, 3, 3, device="cuda").contiguous(memory_format=CL)
for _ in range(a.iters):
    if a.pas == "fwd":
        lib.conv3_tap(x, op, a.co, True)
    elif a.pas == "dgrad":
        lib.conv3_tap(dy, wf, a.c, False)
    elif a.pas == "wgrad_tuned":        # the shipped tuner's pick (implicit-GEMM k_gemm)
        CV.conv_wgrad(dy, x, tuple(w.shape), 1, 1, out=dw)
    elif a.pas == "fwd_tuned":
        CV.conv_fwd(x, w, 1, 1, stats=True)
    else:
        lib.conv3_tap_wgrad(dy, x, dw, True)
torch.cuda.synchronize()
print("done")
