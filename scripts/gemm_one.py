#!/usr/bin/env python
"""Run one MFMA GEMM problem repeatedly (for rocprofv3 counter passes on a single kernel).
usage: gemm_one.py M N K tile [layout fwd|dgrad|wgrad] [iters] [splits]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

M, N, K, tile = (int(v) for v in sys.argv[1:5])
lay = sys.argv[5] if len(sys.argv) > 5 else "fwd"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
splits = int(sys.argv[7]) if len(sys.argv) > 7 else 1
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
if lay == "fwd":
    run = lambda: G.gemm_ex(a, K, True, w, K, True, M, N, K, tile=tile)  # noqa: E731
elif lay == "dgrad":
    wt = w.t().contiguous()
    run = lambda: G.gemm_ex(a, K, True, wt, N, False, M, N, K, tile=tile)  # noqa: E731
else:
    at, wt = a.t().contiguous(), w.t().contiguous()
    run = lambda: G.gemm_ex(at, M, False, wt, N, False, M, N, K, tile=tile, out_bf16=False,  # noqa: E731
                            splits=splits)
for _ in range(iters):
    run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
run()
e.record()
e.synchronize()
ms = s.elapsed_time(e)
print(f"M{M} N{N} K{K} tile{tile} {lay}: {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.0f} TF/s")
