"""MFMA GEMM vs hipBLASLt (torch.mm) on the model shapes (bf16, fp32 accumulate)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from layer_wise_aaai20_amd.ops import gemm as G


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


shapes = [("vgg fc0", 512, 4096, 25088), ("vgg fc1", 512, 4096, 4096), ("alex fc", 512, 4096, 4096),
          ("r50 fc", 256, 1000, 2048), ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
          ("1x1 l1", 802816, 64, 256), ("1x1 l3", 50176, 1024, 256), ("1x1 l4", 12544, 2048, 512)]
for name, M, N, K in shapes:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    fl = 2 * M * N * K
    t = {}
    t["fwd lw"] = bench(lambda: G.linear_fwd(x, w))
    t["fwd bl"] = bench(lambda: torch.mm(x, w.t()))
    t["dgr lw"] = bench(lambda: G.linear_dgrad(dy, w))
    t["dgr bl"] = bench(lambda: torch.mm(dy, w))
    t["wgr lw"] = bench(lambda: G.linear_wgrad(dy, x))
    t["wgr bl"] = bench(lambda: torch.mm(dy.t(), x))
    print(f"{name:8s} M{M:7d} N{N:5d} K{K:5d} | " + " ".join(
        f"{k} {v:7.3f}ms {fl / v / 1e9:6.0f}TF" for k, v in t.items()), flush=True)
