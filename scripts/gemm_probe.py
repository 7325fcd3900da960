"""Run one GEMM configuration repeatedly (for rocprofv3 counter collection).
usage: gemm_probe.py M N K a_kc b_kc tile [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
a_kc, b_kc = sys.argv[4] == "1", sys.argv[5] == "1"
tile = sys.argv[6]
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
A = torch.randn(M * K, device="cuda").bfloat16()
B = torch.randn(N * K, device="cuda").bfloat16()
for _ in range(iters):
    G.gemm_ex(A, K if a_kc else M, a_kc, B, K if b_kc else N, b_kc, M, N, K, tile=tile)
torch.cuda.synchronize()
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
s.record()
for _ in range(iters):
    G.gemm_ex(A, K if a_kc else M, a_kc, B, K if b_kc else N, b_kc, M, N, K, tile=tile)
e.record()
torch.cuda.synchronize()
print(f"{M}x{N}x{K} {tile}: {s.elapsed_time(e) / iters:.4f} ms")
